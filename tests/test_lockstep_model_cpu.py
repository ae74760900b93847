"""workloads.lockstep_cost: the timing model of the reference's per-pass lockstep on the packer's
own rank assignment (small sizes here; DESIGN.md §6 quotes the 8-rank C3 figures)."""

from pipelinerl_amd import workloads


def test_lockstep_model_orders_its_times():
    r = workloads.lockstep_cost("c3", ranks=4, samples_per_rank=8, seed=3)
    assert r["passes"] >= 1 and len(r["sentinels_per_rank"]) == 4
    ms = r["ms"]
    assert ms["balanced"] <= ms["free"] <= ms["forward_then_exchange"] <= ms["exchange_then_forward"] <= ms["full_pass"]
    assert ms["free"] <= ms["loop"] <= ms["exchange_then_forward"]
    assert 0 < r["efficiency"]["full_pass"] <= r["efficiency"]["free"] <= 1
    # one rank: nothing to wait for
    one = workloads.lockstep_cost("c3", ranks=1, samples_per_rank=8, seed=3)["ms"]
    assert abs(one["full_pass"] - one["balanced"]) < 1e-6 and abs(one["forward_then_exchange"] - one["balanced"]) < 1e-6
    assert abs(one["loop"] - one["balanced"]) < 1e-6

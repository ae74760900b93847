"""The N = 1 bound on C3's data-parallel scaling (trainer_probe.projected_dp_efficiency, bench.py
dp_scaling): C3's efficiency at N = lockstep efficiency (workloads.LOCKSTEP_EFFICIENCY) x (1 -
exposed all-reduce ms / the real 4096-sample step), the exposed time measured at N = 1 with an
emulated ring all-reduce (trainer_probe.EmulatedRingBuckets)."""

import pytest


def test_projection_arithmetic():
    from pipelinerl_amd.trainer_probe import projected_dp_efficiency

    # 512 micro-batches of 350 ms per rank + a 40 ms optimizer tail + 20 ms exposed all-reduce
    r = projected_dp_efficiency(0.95, 20.0, 350.0, 512.0, 40.0)
    step = 512 * 350.0 + 40.0 + 20.0
    assert r["step_ms"] == pytest.approx(step, abs=0.05)
    assert r["allreduce_efficiency"] == pytest.approx(1 - 20.0 / step, abs=1e-6)
    assert r["projected_efficiency"] == pytest.approx(0.95 * (1 - 20.0 / step), abs=1e-4)
    assert projected_dp_efficiency(1.0, 0.0, 1.0, 1.0, 0.0)["projected_efficiency"] == 1.0
    # an exposed all-reduce as long as the rest of the step halves the all-reduce efficiency
    assert projected_dp_efficiency(1.0, 100.0, 50.0, 2.0, 0.0)["allreduce_efficiency"] == 0.5


def test_lockstep_table_covers_the_scaling_run():
    from pipelinerl_amd.workloads import LOCKSTEP_EFFICIENCY

    t = LOCKSTEP_EFFICIENCY["c3"]
    assert set(t) >= {2, 4, 8}
    assert all(0.5 < t[n] <= 1.0 for n in t)
    assert t[2] >= t[4] >= t[8]  # more ranks, more sentinel passes and coupling


def test_ring_arms_bytes():
    """Each arm moves 2(N-1)/N of the gradient bytes per GPU."""
    from pipelinerl_amd.trainer_probe import RING_ARMS

    assert RING_ARMS["n8_1link"][:2] == (8, 153.0) and RING_ARMS["n4_1link"][:2] == (4, 153.0)
    S = 15.23e9
    assert 2 * (8 - 1) / 8 * S == pytest.approx(26.65e9, rel=1e-3)
    assert RING_ARMS["n8_7links"][1] == pytest.approx(7 * 153.0)


def test_dp_probe_cpu_ignores_emulation():
    """The emulation needs a HIP device; on CPU (gloo rehearsals) the probe runs without it, and a
    value-head model takes the same probe (its value_loss_coef set)."""
    import torch

    from cpu_rl_step import cpu_rl_step
    from loop_helpers import rollouts
    from pipelinerl_amd import workloads
    from pipelinerl_amd.trainer_probe import RING_ARMS, dp_step_probe
    from test_split_pipeline_cpu import _tiny

    data = rollouts(4, 4, seed=0)
    batches = [b for _, b in workloads.pack(data, 48, len(data)) if not b.sentinel][:2]
    r = dp_step_probe("c3", steps=1, warmup=1, device=torch.device("cpu"), samples_per_step=64, batches=batches,
                      model=_tiny().float(), step_fn=cpu_rl_step, emulate=RING_ARMS)
    assert "allreduce_emulated" not in r and r["ms_per_step_local"] > 0

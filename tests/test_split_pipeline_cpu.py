"""The split trainer / actor probe (trainer_probe.split_pipeline_probe, BASELINE configs[3]) on
CPU gloo: W - A trainer ranks train data-parallel on a tiny bf16 Qwen2 with the test-only torch
loss while trainer rank 0 broadcasts every step's weights to A actor ranks.  Checks the group
layout, that every update is received (the actors end with the trainer's weights, bit-exact)
and that the report is complete."""

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _tiny():
    from transformers import Qwen2Config, Qwen2ForCausalLM

    torch.manual_seed(0)
    cfg = Qwen2Config(vocab_size=96, hidden_size=32, intermediate_size=64, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                      tie_word_embeddings=True)
    return Qwen2ForCausalLM(cfg).to(torch.bfloat16)


def _run(rank, port, world, actors, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from cpu_rl_step import cpu_rl_step
    from pipelinerl_amd.trainer_probe import TrainerStep, split_pipeline_probe
    from test_weight_update_cpu import TorchFlatPacker

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cpu")
    holder = {}

    def make_trainer(group):
        ts = TrainerStep(tokens=64, seq=32, prompt=8, micro_batches=2, device=dev, group=group, model=_tiny(),
                         step_fn=cpu_rl_step, vocab=96)
        holder["model"] = ts.model
        return ts

    def make_actor():
        m = _tiny()
        for p in m.parameters():
            p.data.zero_()
        holder["model"] = m
        return m

    res = split_pipeline_probe(actors, steps=2, warmup=1, device=dev, bucket_bytes=4096,
                               make_trainer=make_trainer, make_actor_module=make_actor, packer=TorchFlatPacker())
    params = {n: p.detach().clone() for n, p in holder["model"].named_parameters()}
    torch.save({"res": res, "params": params}, Path(out) / f"r{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,actors", [(2, 1), (4, 2), (8, 4)])  # (8, 4): C4 on one node
def test_split_pipeline_gloo(tmp_path, world, actors):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), world, actors, str(tmp_path)), nprocs=world, join=True)
    got = [torch.load(tmp_path / f"r{r}.pt") for r in range(world)]
    n_tr = world - actors
    r0 = got[0]["res"]
    assert all(g["res"] == r0 for g in got)  # one report, on every rank
    assert r0["trainers"] == n_tr and r0["actors"] == actors and r0["updates"] == 3
    assert r0["broadcast_latency_ms"] > 0 and 0.0 <= r0["hidden_frac"] <= 1.0
    assert r0["broadcast_bytes"] == sum(2 * p.numel() for p in got[0]["params"].values())
    # the census of both groups, as trainer rank 0 saw it: the DP group and the actor group (1 + actors)
    g = r0["groups"]
    assert g["split_dp"]["reported"] == g["split_dp"]["participants"] == n_tr
    assert g["actor"]["reported"] == g["actor"]["participants"] == 1 + actors
    for r in range(n_tr, world):  # actors hold the trainer's last snapshot exactly
        for n, p in got[0]["params"].items():
            assert torch.equal(got[r]["params"][n], p), (r, n)
    for r in range(1, n_tr):  # DP replicas stay identical
        for n, p in got[0]["params"].items():
            assert torch.equal(got[r]["params"][n], p), (r, n)


def _fsdp_run(rank, port, world, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from cpu_rl_step import cpu_rl_step
    from pipelinerl_amd.trainer_probe import TrainerStep

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ts = TrainerStep(tokens=64, seq=32, prompt=8, micro_batches=2, device=torch.device("cpu"), model=_tiny().float(),
                     step_fn=cpu_rl_step, vocab=96, fsdp=True, kl_coef=0.001)
    assert ts.cfg.kl_coef == 0.001 and ts.grads is None
    assert not torch.equal(ts.batches[0].ref_logprobs, ts.batches[0].old_logprobs)  # KL term is live
    sec = ts.timed(2, 1)
    full = {n: p.detach().full_tensor().clone() for n, p in ts.model.named_parameters()}
    torch.save({"sec": sec, "params": full}, Path(out) / f"f{rank}.pt")
    dist.destroy_process_group()


def test_fsdp_trainer_step_gloo(tmp_path):
    """The configs[4] probe's step (TrainerStep(fsdp=True), KL on) on gloo world 2: runs, and the
    gathered parameters agree on both ranks after three optimizer steps."""
    from test_weight_update_cpu import free_port

    mp.spawn(_fsdp_run, args=(free_port(), 2, str(tmp_path)), nprocs=2, join=True)
    a, b = (torch.load(tmp_path / f"f{r}.pt") for r in range(2))
    assert a["sec"] > 0 and b["sec"] > 0
    for n, p in a["params"].items():
        assert torch.equal(p, b["params"][n]), n


def _dp_run(rank, port, world, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from cpu_rl_step import cpu_rl_step
    from loop_helpers import rollouts
    from pipelinerl_amd import workloads
    from pipelinerl_amd.trainer_probe import dp_step_probe

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data = rollouts(4, 4, seed=rank)  # a different sample per rank, as the probe draws them
    batches = [b for _, b in workloads.pack(data, 48, len(data)) if not b.sentinel][:3]
    res = dp_step_probe("c3", steps=2, warmup=1, device="cpu", samples_per_step=64, batches=batches,
                        model=_tiny().float(), step_fn=cpu_rl_step)
    torch.save(res, Path(out) / f"dp{rank}.pt")
    dist.destroy_process_group()


def test_c3_dp_probe_gloo(tmp_path):
    """bench.py's c3_dp probe (trainer_probe.dp_step_probe) on gloo world 2: the replica's step
    alone, the DP step with the bucketed all-reduce, the all-reduce alone; one consistent report
    on every rank, with the extrapolation to the config's samples-per-step."""
    from test_weight_update_cpu import free_port

    mp.spawn(_dp_run, args=(free_port(), 2, str(tmp_path)), nprocs=2, join=True)
    a, b = (torch.load(tmp_path / f"dp{r}.pt") for r in range(2))
    for k in ("ms_per_step_local", "allreduce_bytes", "tokens_per_rank_step", "samples_per_rank_step", "world"):
        assert a[k] == b[k], k
    assert a["world"] == 2 and a["micro_batches_per_rank"] == 3
    assert a["ms_per_step_local"] > 0 and a["ms_per_step_dp"] > 0 and a["allreduce_alone_ms"] > 0
    assert a["allreduce_bytes"] == sum(p.numel() * 4 for p in _tiny().parameters())
    assert a["overlap"] is not None and 0.0 <= a["overlap"] <= 1.0
    ex = a["extrapolated"]
    assert ex["samples_per_step"] == 64 and ex["micro_batches_per_rank"] > 0 and ex["tokens_per_s_per_gpu"] > 0

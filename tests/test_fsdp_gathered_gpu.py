"""FSDP layers kept gathered from forward to backward (finetune.fsdp_keep_gathered_layers:
finetune/recompute.py plan_fsdp_gathering -> finetune/sharding.py shard_model), at config C5's
layer shapes (Qwen2.5-32B: H 5120, 40 / 8 heads, I 27 648, V 152 064) with 4 decoder layers, on
two ranks sharing cuda:0 through gloo (as tests/test_fsdp_32b_gpu.py): correctness and peak memory
only — one GPU says nothing about the all-gather time saved.

For R = 0 (FSDP2's default: every layer resharded after its forward, gathered again for its
backward) and R = 4 (every layer stays gathered), each rank runs two packed 4 096-token rl_step
micro-batches with an AdamW step after each (the reference's C5 step shape, kl_coef 0.001):
  1. the first step's gradient shards are bit-identical for both R (the same all-gathered values
     feed the same deterministic kernels);
  2. the steady-state peak (the second step) grows by at most the plan's gathered bytes
     (R x a layer's rounded unsharded parameters) and by at least one layer (at the start of the
     backward R = 4 holds four layers, R = 0 the current and the prefetched one);
  3. the plan's estimate for R = 4 (terms without the fixed headroom, gathered bytes included)
     covers that peak.
"""

from __future__ import annotations

import gc
import json
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu
T, SEQ, PROMPT, LAYERS = 4096, 1024, 128, 4


def _run(rank: int, port: int, tmp: str):
    import time

    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "4"
    import torch.distributed as dist

    from pipelinerl_amd.finetune.optim import clip_grad_norm, get_optimizer
    from pipelinerl_amd.finetune.recompute import gathered_layer_bytes, plan_gradient_checkpointing
    from pipelinerl_amd.finetune.rl import rl_step
    from pipelinerl_amd.finetune.sharding import shard_model
    from pipelinerl_amd.trainer_probe import QWEN, packed_batch, qwen2_model, rl_config
    from test_fsdp_32b_gpu import _digest, _offset

    t0 = time.time()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    batch = packed_batch(T, SEQ, PROMPT, QWEN["32b"]["vocab_size"], dev, seed=100 + rank, ref_noise=True)
    cfg = rl_config(2 * (T // SEQ), kl_coef=0.001)
    out: dict = {}
    for R in (0, LAYERS):
        torch.manual_seed(0)
        model = shard_model(qwen2_model("32b", dev, layers=LAYERS), keep_gathered=R)
        opt = get_optimizer("adamw_torch", model, 1e-6, 0.01)

        def step():
            loss, stats = rl_step(model, batch, 0, 10, cfg, defer_stats=True)
            loss.backward()
            stats.resolve()

        step()
        digest = {n: _digest(p.grad.to_local(), _offset(p)) for n, p in model.named_parameters()}
        clip_grad_norm(model.parameters(), 0.3, opt)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
        base = int(torch.cuda.memory_allocated(dev))
        t1 = time.time()
        step()
        clip_grad_norm(model.parameters(), 0.3, opt)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        peak = int(torch.cuda.max_memory_allocated(dev))
        args = {"gradient_checkpointing": True, "gradient_checkpointing_policy": "auto", "seq_length": T,
                "rl": {"lm_head_chunk_rows": 65536}, "fsdp_keep_gathered_layers": R}
        plan = plan_gradient_checkpointing(args, model, dev, shard_world=2)
        out[str(R)] = {"digest": digest, "peak_bytes": peak, "base_bytes": base, "plan": plan.as_dict(),
                       "gathered_bytes": plan.gathered_bytes, "step_s": time.time() - t1,
                       "layer_bytes": gathered_layer_bytes(model),
                       "estimate_bytes": plan.state_bytes + plan.activation_bytes + plan.logits_bytes +
                       plan.buffer_bytes + plan.gathered_bytes}
        print(f"[rank {rank} +{time.time() - t0:.0f}s] R={R} peak {peak / 1e9:.2f} GB", flush=True)
        del model, opt
        gc.collect()  # FSDP's module <-> state cycles: else the previous model stays on the device
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    with open(Path(tmp) / f"rank{rank}.json", "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_c5_shapes_layers_kept_gathered(tmp_path):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(2)]
    # a layer's unsharded bytes after the allocator rounding in force in the ranks (devalloc.py)
    per = r[0]["0"]["layer_bytes"]
    raw = (2 * 5120 * 5120 + 2 * 1024 * 5120 + 3 * 27648 * 5120 + 5120 + 2 * 1024 + 2 * 5120) * 2
    assert raw <= per <= 1.1 * raw, (per, raw)
    summary = {f"rank{i}": {R: {"peak_gb": x[R]["peak_bytes"] / 1e9, "estimate_gb": x[R]["estimate_bytes"] / 1e9,
                                "step_s": round(x[R]["step_s"], 2)} for R in x} for i, x in enumerate(r)}
    print(json.dumps({"layer_gb": per / 1e9, "summary": summary}))
    g = str(LAYERS)
    for i, x in enumerate(r):
        bad = [n for n in x["0"]["digest"] if x["0"]["digest"][n] != x[g]["digest"][n]]
        assert not bad, (i, bad[:5])
        assert x[g]["gathered_bytes"] == LAYERS * per and x["0"]["gathered_bytes"] == 0
        grow = x[g]["peak_bytes"] - x["0"]["peak_bytes"]
        assert per <= grow <= x[g]["gathered_bytes"], (i, grow / 1e9, per / 1e9)
        assert x[g]["peak_bytes"] <= x[g]["estimate_bytes"], (i, summary)


def _probe_rank(rank: int, port: int, tmp: str):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "4"
    import torch.distributed as dist

    from pipelinerl_amd.trainer_probe import fsdp_step_probe

    torch.cuda.set_device(0)
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    r = fsdp_step_probe("32b", tokens=2048, micro_batches=1, steps=1, warmup=0, device=torch.device("cuda:0"),
                        layers=2, keep_gathered="plan")
    if rank == 0:
        (Path(tmp) / "probe.json").write_text(json.dumps(r))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_fsdp_probe_applies_the_plan(tmp_path):
    """bench.py's fsdp_32b_kept_gathered probe path: fsdp_step_probe(keep_gathered="plan") sizes R
    with the loop's plan on the sharded model and keeps that many layers gathered (2 of 2 here)."""
    from test_weight_update_cpu import free_port

    mp.spawn(_probe_rank, args=(free_port(), str(tmp_path)), nprocs=2, join=True)
    r = json.loads((tmp_path / "probe.json").read_text())
    print(json.dumps(r))
    assert r["kept_gathered_layers"] == 2 and r["plan"]["gathered_layers"] == 2, r
    assert r["ms_per_optimizer_step"] > 0 and r["tokens_per_s"] > 0

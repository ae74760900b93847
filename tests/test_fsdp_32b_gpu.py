"""Config C5's sharded trainer at its own layer shapes (BASELINE.json configs[4]; the reference's
FSDP path, /root/reference/pipelinerl/finetune_loop.py:222-232 and :369-380).

Qwen2.5-32B dimensions (H 5120, 40 / 8 heads of 128, I 27 648, V 152 064, untied lm_head) with 2 of
its 64 decoder layers, the patched HIP model ops, FSDP2 (finetune/sharding.py) over two ranks that
share cuda:0 through gloo (RCCL needs one GPU per rank): FSDP really frees each layer's unsharded
parameters after the forward and gathers them again for the backward.  Each rank trains one packed
4 096-token micro-batch (4 rollouts x 1 024, 128-token prompts) through rl_step with the KL term on
(kl_coef 0.001, ref = old + N(0, 0.05²) on the label tokens).

  1. gradients: the sharded (reduce-scattered, mean over the ranks) gradient of every parameter
     equals one unsharded model's gradient of the mean of both ranks' losses, per tensor within
     the bf16 GEMM bar (relative norm 2e-2; the unsharded side runs the label-row lm_head, the
     sharded side the full-logits loss head);
  2. weight update: after the optimizer step, rank 0's WeightUpdateManager snapshot (bucketed
     all-gathers, HIP flatten) is broadcast to an actor held by rank 1, once per transport
     (per_tensor into a trainer-layout actor, bucketed into vLLM's fused qkv_proj / gate_up_proj
     layout) and every received region is bit-identical to the trainer's gathered parameter;
  3. the gradient-checkpointing plan (finetune/recompute.py, ``gradient_checkpointing_policy:
     auto`` against conf/finetune/base.yaml:44-45): its estimate for this model at 4 096 tokens,
     without the fixed headroom (5 % of the device + 4 GiB), is >= the measured peak of the
     steady-state step (torch.cuda.max_memory_allocated over the second step's forward + backward +
     AdamW step, the moments resident, no recompute) and <= 1.3 x it.
"""

from __future__ import annotations

import json
import math
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu
T, SEQ, PROMPT, LAYERS = 4096, 1024, 128, 2
GRAD_REL = 2e-2


def _batch(rank: int):
    from pipelinerl_amd.trainer_probe import QWEN, packed_batch

    return packed_batch(T, SEQ, PROMPT, QWEN["32b"]["vocab_size"], torch.device("cuda:0"), seed=100 + rank,
                        ref_noise=True)


def _cfg():
    from pipelinerl_amd.trainer_probe import rl_config

    return rl_config(2 * (T // SEQ), kl_coef=0.001)


def _run(rank: int, port: int, tmp: str):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "4"
    import torch.distributed as dist

    from pipelinerl_amd.actor import StandaloneWorker
    from pipelinerl_amd.finetune.optim import clip_grad_norm, get_optimizer
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing
    from pipelinerl_amd.finetune.rl import rl_step
    from pipelinerl_amd.finetune.sharding import shard_model
    from pipelinerl_amd.trainer_probe import qwen2_model
    from pipelinerl_amd.weight_update import WeightUpdateManager, WeightUpdateRequest, parameters_info

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    # gloo for CUDA tensors too: FSDP's device mesh would otherwise open an RCCL group, which
    # cannot span two ranks on one GPU
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    out: dict = {}
    model = shard_model(qwen2_model("32b", dev, layers=LAYERS))
    opt = get_optimizer("adamw_torch", model, 1e-6, 0.01)
    batch = _batch(rank)

    def step():
        loss, stats = rl_step(model, batch, 0, 10, _cfg(), defer_stats=True)
        loss.backward()
        st = stats.resolve()
        assert st["kl"] > 0 and st["num_output_tokens_sum"] == (T // SEQ) * (SEQ - PROMPT)

    # step 1: the sharded gradients of the initial weights, gathered (collective) to the host
    step()
    grads = {}
    for n, p in model.named_parameters():
        full = p.grad.full_tensor()
        if rank == 0:
            grads[n] = full.float().cpu()
        del full
    clip_grad_norm(model.parameters(), 0.3, opt)
    opt.step()
    opt.zero_grad(set_to_none=True)
    # step 2, the steady state (AdamW moments resident through the backward): its peak memory
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    out["base_bytes"] = int(torch.cuda.memory_allocated(dev))
    step()
    clip_grad_norm(model.parameters(), 0.3, opt)
    opt.step()
    opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    out["peak_bytes"] = int(torch.cuda.max_memory_allocated(dev))
    args = {"gradient_checkpointing": True, "gradient_checkpointing_policy": "auto", "seq_length": T,
            "rl": {"lm_head_chunk_rows": 65536}}
    plan = plan_gradient_checkpointing(args, model, dev, shard_world=2)
    out["plan"] = plan.as_dict()
    out["estimate_bytes"] = plan.state_bytes + plan.activation_bytes + plan.logits_bytes + plan.buffer_bytes

    # ---- weight update: rank 0 trains and sends, rank 1 also holds the actor --------------------
    named = list(model.named_parameters())
    infos = parameters_info(named)
    checks = {}
    for version, (transport, layout) in enumerate((("per_tensor", "trainer"), ("bucketed", "vllm")), start=1):
        wum = WeightUpdateManager([], model, None, dist.group.WORLD, transport=transport, bucket_bytes=256 << 20,
                                  overlap=True, is_main=rank == 0, write_message=lambda s, m: None)
        if rank == 1:
            actor = qwen2_model("32b", dev, fused_ops=False, layers=LAYERS)
            with torch.no_grad():
                for p in actor.parameters():
                    p.zero_()
            worker = StandaloneWorker(actor, rank=0, device=dev, layout=layout)
            worker.process_group = dist.group.WORLD
        wum.send_weight_update(version)  # every rank takes part in the bucketed all-gathers
        if rank == 1:
            worker.receive_weight_update(WeightUpdateRequest(
                version=version, parameters_info=infos, transport=transport,
                bucket_bytes=256 << 20 if transport == "bucketed" else 0))
        else:
            wum.wait()
        wum.close()
        torch.cuda.synchronize()
        equal, n = 0, 0
        for name, p in named:
            full = p.detach().full_tensor().to(torch.bfloat16)  # collective: both ranks
            if rank == 1:
                got = worker.model_runner.model.direct_target(name, tuple(full.shape))
                n += 1
                equal += int(got is not None and torch.equal(got, full))
        if rank == 1:
            checks[transport] = {"equal": equal, "tensors": n, "layout": layout}
            del worker, actor
            torch.cuda.empty_cache()
    out["weight_update"] = checks

    if rank == 0:  # unsharded model, same init: gradient of the mean of both ranks' losses
        ref = qwen2_model("32b", dev, layers=LAYERS)
        total = None
        for r in range(2):
            lo, _ = rl_step(ref, _batch(r), 0, 10, _cfg())
            total = lo * 0.5 if total is None else total + lo * 0.5
        total.backward()
        errs = {}
        for name, p in ref.named_parameters():
            r, g = p.grad.float().cpu().double(), grads[name].double()
            rr = float((r * r).sum())
            errs[name] = math.sqrt(float(((g - r) ** 2).sum()) / rr) if rr > 0 else float(g.abs().max())
        out["grad_rel_err"] = errs
        del ref
    with open(Path(tmp) / f"rank{rank}.json", "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_c5_32b_shapes_fsdp_grads_snapshot_and_memory_plan(tmp_path):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = json.loads((tmp_path / "rank0.json").read_text())
    r1 = json.loads((tmp_path / "rank1.json").read_text())
    errs = r0["grad_rel_err"]
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    mem = {r: (d["peak_bytes"] / 1e9, d["estimate_bytes"] / 1e9) for r, d in (("rank0", r0), ("rank1", r1))}
    print(json.dumps({"worst_grad_rel_err": worst, "tensors": len(errs), "peak_vs_estimate_gb": mem,
                      "plan": r1["plan"], "weight_update": r1["weight_update"]}))
    assert len(errs) == 3 + LAYERS * 12, len(errs)  # embed, norm, lm_head + 12 per decoder layer
    assert worst[0][1] <= GRAD_REL, worst
    for transport, c in r1["weight_update"].items():
        assert c["equal"] == c["tensors"] == len(errs), (transport, c)
    for r, (peak, est) in mem.items():
        assert peak <= est <= 1.3 * peak, (r, peak, est, r1["plan"])

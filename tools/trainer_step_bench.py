"""Trainer-step and loss-head comparisons on one MI355X (measurement tool).

  --mode loss     fused HIP loss head vs the reference's ATen op chain (tools/aten_rl_step.py)
                  on the same bf16 logits, fwd+bwd per packed micro-batch
  --mode trainer  full trainer micro-batch step on a Qwen2.5-shaped model (random init, bf16,
                  prl_varlen attention): forward, loss head, backward, clip, fused AdamW.  Loss heads:
                  fused (HIP kernel on full logits), fused_head (label-row chunked lm_head + HIP
                  kernel, RLConfig.fused_lm_head), aten (the reference's op chain)
Prints one JSON line per measured configuration.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
import types
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from pipelinerl_amd.trainer_probe import QWEN, packed_batch  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def rl_cfg(fused_head: bool = False, chunk: int = 65536):
    from pipelinerl_amd.finetune.rl import RLConfig

    return RLConfig(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, final_kl_coef=0.0, clamp_log_ratio_ref_new_value=5,
                    batch_size=4096, fused_lm_head=fused_head, lm_head_chunk_rows=chunk)


def mode_loss(a):
    from aten_rl_step import aten_loss_head
    from pipelinerl_amd.finetune.rl import rl_step

    V = a.vocab
    batch = packed_batch(a.tokens, a.seq, a.prompt, V, "cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    logits = (torch.randn((1, a.tokens, V), generator=g, device="cuda") * 3).to(torch.bfloat16)
    model = types.SimpleNamespace(config=None)
    cfg = rl_cfg()
    out = {}
    for name in a.loss.split(","):
        lg = logits.clone().requires_grad_(True)

        def step():
            lg.grad = None
            if name == "fused":
                m = types.SimpleNamespace(logits=lg)
                loss, _ = rl_step(lambda **kw: m, batch, 0, 100, cfg)
            else:
                loss, _ = aten_loss_head(lg, batch, cfg)
            loss.backward()

        torch.cuda.reset_peak_memory_stats()
        dt = timed(step, a.steps, a.warmup)
        out[name] = {"ms": round(dt * 1e3, 3), "tokens_per_s": round(a.tokens / dt, 1),
                     "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2)}
        del lg
        torch.cuda.empty_cache()
    print(json.dumps({"mode": "loss", "T": a.tokens, "V": V, "dtype": "bf16", "results": out}), flush=True)


def mode_trainer(a):
    from aten_rl_step import aten_loss_head
    from pipelinerl_amd.finetune.attention import packed_kwargs
    from pipelinerl_amd.finetune.optim import get_optimizer
    from pipelinerl_amd.finetune.rl import rl_step

    from pipelinerl_amd.trainer_probe import qwen2_model

    shapes = QWEN[a.model]
    model = qwen2_model(a.model, torch.device("cuda"), a.grad_ckpt, fused_ops=not a.eager_ops)
    opt = get_optimizer("adamw_torch", model, 1e-6, 0.01)
    batch = packed_batch(a.tokens, a.seq, a.prompt, shapes["vocab_size"], "cuda")
    out = {}
    for name in a.loss.split(","):
        cfg = rl_cfg(name == "fused_head", a.chunk)

        def step():
            if name in ("fused", "fused_head"):
                loss, _ = rl_step(model, batch, 0, 100, cfg)
            else:
                o = model(input_ids=batch.input_ids, position_ids=batch.position_ids,
                          **packed_kwargs(batch, "cuda"))
                loss, _ = aten_loss_head(o.logits, batch, cfg)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 0.3)
            opt.step()
            opt.zero_grad(set_to_none=True)

        torch.cuda.reset_peak_memory_stats()
        try:
            dt = timed(step, a.steps, a.warmup)
            out[name] = {"ms_per_micro_batch_step": round(dt * 1e3, 2), "tokens_per_s": round(a.tokens / dt, 1),
                         "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2)}
        except torch.OutOfMemoryError as e:
            out[name] = {"oom": str(e)[:200]}
        opt.zero_grad(set_to_none=True)
        torch.cuda.empty_cache()
    print(json.dumps({"mode": "trainer", "model": f"Qwen2.5-{a.model} shapes (random init)", "T": a.tokens,
                      "seq": a.seq, "grad_ckpt": a.grad_ckpt, "fused_model_ops": not a.eager_ops,
                      "results": out}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["loss", "trainer"], default="loss")
    ap.add_argument("--model", choices=list(QWEN), default="1.5b")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--loss", default="fused,aten")
    ap.add_argument("--grad-ckpt", action="store_true")
    ap.add_argument("--eager-ops", action="store_true", help="HF eager RMSNorm / SwiGLU / RoPE (no model_ops patch)")
    ap.add_argument("--chunk", type=int, default=65536, help="lm_head_chunk_rows for --loss fused_head")
    a = ap.parse_args()
    mode_loss(a) if a.mode == "loss" else mode_trainer(a)

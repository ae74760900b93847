"""Throughput of the fp32-master AdamW step (csrc/adamw.hip prl_adamw_master_step via PrlAdamW) on
a model's full parameter list (Qwen2.5 shapes, random values): bf16 parameters in one flat buffer as
the trainer re-homes them, bf16 gradients, fp32 master / exp_avg / exp_avg_sq, the clip coefficient
folded in.  Algorithmic bytes: 28 per parameter (read g 2 + master, m, v 12; write master, m, v 12 +
p 2).  Prints one JSON line; `--bf16` times the pure-bf16 step (14 B / parameter) for comparison.

    python tools/adamw_master_bench.py --model 7b --steps 10
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="7b")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--bf16", action="store_true", help="pure-bf16 state (no masters)")
    a = ap.parse_args()
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.finetune.optim import clip_grad_norm, get_optimizer
    from pipelinerl_amd.trainer_probe import QWEN
    from pipelinerl_amd.weight_update import rehome_parameters

    dev = torch.device("cuda")
    with torch.device(dev):
        model = AutoModelForCausalLM.from_config(Qwen2Config(**QWEN[a.model]), dtype=torch.bfloat16)
    rehome_parameters(model)
    params = [p for p in model.parameters()]
    n = sum(p.numel() for p in params)
    g = torch.Generator(device=dev).manual_seed(0)
    for p in params:
        p.grad = (torch.randn(p.shape, generator=g, device=dev) * 1e-3).to(torch.bfloat16)
    opt = get_optimizer("adamw_torch", model, 5e-7, 0.01, master_weights=not a.bf16)
    for _ in range(2):  # warm-up: state allocation, first launches
        clip_grad_norm(params, 0.3, opt)
        opt.step()
    torch.cuda.synchronize()
    times = []
    for _ in range(a.steps):
        clip_grad_norm(params, 0.3, opt)  # the norm runs outside the timed step
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        opt.step()
        e.record()
        torch.cuda.synchronize()
        times.append(s.elapsed_time(e) / 1e3)
    per = 14 if a.bf16 else 28
    t = sorted(times)[len(times) // 2]
    print(json.dumps({"model": a.model, "params": n, "state": "bf16" if a.bf16 else "fp32_master",
                      "bytes_per_param": per, "step_ms_median": round(t * 1e3, 3),
                      "step_ms_min": round(min(times) * 1e3, 3), "achieved_gbps": round(per * n / t / 1e9, 1),
                      "frac_of_8tbps": round(per * n / t / 8e12, 4)}))


if __name__ == "__main__":
    main()

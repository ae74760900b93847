"""The fused loss head with bf16 logits (DeepSpeed regime, the resident kernel) and fp32 logits
(Accelerate mixed precision upcasts the logits: the streaming kernel, whose gradient pass
re-reads the row) at the same packed micro-batch; algorithmic bytes = logits read once + dlogits
written once (measurement tool).

    python tools/loss_dtype_bench.py [--tokens 65536] [--vocab 151936]
"""

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=151936)
    a = ap.parse_args()
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    dev = torch.device("cuda", 0)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    for dt in (torch.bfloat16, torch.float32):
        logits, fields = bench.make_workload(a.tokens, a.vocab, 2048, 256, 1234, dev)
        if dt == torch.float32:
            logits = logits.detach().float().requires_grad_(True)
        times = []
        for i in range(8):
            logits.grad = None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            loss, _, _ = grpo_loss(logits, fields, params)
            e1.record()
            loss.backward()
            torch.cuda.synchronize()
            if i >= 2:
                times.append(e0.elapsed_time(e1))
        ms = sum(times) / len(times)
        b = logits.element_size()
        alg = 2.0 * a.tokens * a.vocab * b + 37 * a.tokens
        print(json.dumps({"logits_dtype": str(dt).replace("torch.", ""), "T": a.tokens, "V": a.vocab, "ms": round(ms, 3),
                          "algorithmic_GBps": round(alg / ms / 1e6, 1), "tokens_per_s": round(a.tokens / ms * 1e3, 1)}),
              flush=True)
        del logits, fields, loss
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

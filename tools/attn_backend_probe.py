"""Packed causal attention fwd+bwd on one MI355X, per formulation: torch varlen flash attention
with native GQA (the trainer's path) or with repeated k/v, and batched SDPA (equal-length
rollouts only).  Shapes: Qwen2.5-1.5B attention (12 q heads, 2 kv heads, head dim 128),
T = 16384 packed as 8 x 2048 (and 2 x 8192).  Prints one JSON line per case."""
import json
import time

import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from torch.nn.attention.varlen import varlen_attn


def bench(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def case(T, seq, hq=12, hkv=2, D=128):
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda h: torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16).requires_grad_()  # noqa
    q, k, v = mk(hq), mk(hkv), mk(hkv)
    do = torch.randn((T, hq, D), generator=g, device="cuda").to(torch.bfloat16)
    cu = torch.arange(0, T + 1, seq, dtype=torch.int32, device="cuda")
    rep = hq // hkv
    flops = 3.5 * 4 * (T // seq) * seq * seq * D * hq / 2
    res = {}

    def native():
        varlen_attn(q, k, v, cu, cu, seq, seq, is_causal=True).backward(do)

    def repeated():
        varlen_attn(q, k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1), cu, cu, seq, seq,
                    is_causal=True).backward(do)

    def batched():
        B = T // seq
        qb = q.view(B, seq, hq, D).transpose(1, 2)
        kb = k.view(B, seq, hkv, D).transpose(1, 2)
        vb = v.view(B, seq, hkv, D).transpose(1, 2)
        o = F.scaled_dot_product_attention(qb, kb, vb, is_causal=True, enable_gqa=True)
        o.backward(do.view(B, seq, hq, D).transpose(1, 2))

    def hip_bwd():
        from pipelinerl_amd.finetune.attention import PackedCausalAttention

        PackedCausalAttention.apply(q, k, v, cu, seq, list(range(0, T + 1, seq))).backward(do)

    def fwd_only():
        with torch.no_grad():
            varlen_attn(q, k, v, cu, cu, seq, seq, is_causal=True)

    order = (("varlen_repeated_kv", repeated), ("prl_hip_backward", hip_bwd), ("varlen_gqa_native", native),
             ("sdpa_batched", batched), ("varlen_fwd_only", fwd_only), ("prl_hip_backward_again", hip_bwd),
             ("varlen_repeated_kv_again", repeated))
    for name, fn in order:
        try:
            ms = bench(fn)
            f = flops / 3.5 if name.startswith("varlen_fwd_only") else flops
            res[name] = {"ms": round(ms, 3), "TFLOPs": round(f / (ms * 1e-3) / 1e12, 1)}
        except Exception as e:
            res[name] = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    print(json.dumps({"T": T, "seq": seq, "hq": hq, "hkv": hkv, "D": D, "results": res}), flush=True)


if __name__ == "__main__":
    case(16384, 2048)
    case(16384, 8192)

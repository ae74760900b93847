"""Per-shape throughput of the trainer step's library GEMMs (hipBLASLt via torch) for Qwen2.5
shapes at T tokens: forward Y = X W^T, dgrad dX = dY W, wgrad dW = dY^T X, each timed alone.
Prints one JSON line per (layer, pass)."""
import json
import sys
import time

import torch

T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
model = sys.argv[2] if len(sys.argv) > 2 else "1.5b"
SH = {"1.5b": dict(H=1536, I=8960, KV=256, V=151936), "7b": dict(H=3584, I=18944, KV=512, V=152064)}[model]
H, I, KV, V = SH["H"], SH["I"], SH["KV"], SH["V"]
layers = {"q/o_proj": (H, H), "k/v_proj": (H, KV), "gate/up_proj": (H, I), "down_proj": (I, H), "lm_head": (H, V)}


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


for name, (K, N) in layers.items():
    x = torch.randn((T, K), device="cuda", dtype=torch.bfloat16)
    w = torch.randn((N, K), device="cuda", dtype=torch.bfloat16)
    dy = torch.randn((T, N), device="cuda", dtype=torch.bfloat16)
    flops = 2.0 * T * K * N
    for pas, fn in (("fwd", lambda: torch.nn.functional.linear(x, w)), ("dgrad", lambda: dy @ w),
                    ("wgrad", lambda: dy.t() @ x)):
        sec = bench(fn)
        rec = {"model": model, "T": T, "layer": name, "K": K, "N": N, "pass": pas,
               "ms": round(sec * 1e3, 4), "TFLOPs": round(flops / sec / 1e12, 1)}
        if "--check" in sys.argv:  # max error vs an fp32 GEMM of the same bf16 operands, / max |ref|
            ref = {"fwd": lambda: x.float() @ w.float().t(), "dgrad": lambda: dy.float() @ w.float(),
                   "wgrad": lambda: dy.float().t() @ x.float()}[pas]()
            rec["rel_err"] = float((fn().float() - ref).abs().max() / ref.abs().max())
            del ref
        print(json.dumps(rec), flush=True)
    del x, w, dy
    torch.cuda.empty_cache()

# split-K wgrad: dW = sum_c dY_c^T X_c as one strided batched GEMM + a sum of the fp32 partials
if "--splitk" in sys.argv:
    for name, (K, N) in layers.items():
        if name == "lm_head":
            continue
        x = torch.randn((T, K), device="cuda", dtype=torch.bfloat16)
        dy = torch.randn((T, N), device="cuda", dtype=torch.bfloat16)
        ref = (dy.t().float() @ x.float())
        flops = 2.0 * T * K * N
        for sk in (2, 4, 8, 16):
            def f():
                xs = x.view(sk, T // sk, K)
                ds = dy.view(sk, T // sk, N)
                part = torch.bmm(ds.transpose(1, 2), xs, out_dtype=torch.float32) if hasattr(torch, "bmm") else None
                return part.sum(0).to(torch.bfloat16)
            try:
                sec = bench(f)
                err = float((f().float() - ref).abs().max() / ref.abs().max())
                print(json.dumps({"layer": name, "pass": f"wgrad_splitk{sk}", "ms": round(sec * 1e3, 4),
                                  "TFLOPs": round(flops / sec / 1e12, 1), "rel_err": err}), flush=True)
            except Exception as e:
                print(json.dumps({"layer": name, "pass": f"wgrad_splitk{sk}", "error": str(e)[:200]}), flush=True)
        del x, dy
        torch.cuda.empty_cache()

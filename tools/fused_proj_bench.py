"""Separate vs fused projection GEMMs through prl_gemm (the trainer's GEMM path): q / k / v as three
GEMMs or one over the concatenated [Nq + 2 Nkv, H] weight, gate / up as two or one [2 I, H],
each pass (forward Y = X W^T, dgrad dX = dY W summed over the group, wgrad dW = dY^T X) timed at
T tokens with HIP events.  Decides whether fused projection storage is worth building.

    python tools/fused_proj_bench.py [T] [model]
"""
import json
import sys
from pathlib import Path

import torch

sys.path[:0] = [str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd")]
from pipelinerl_amd import gemm  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
model = sys.argv[2] if len(sys.argv) > 2 else "7b"
SH = {"1.5b": dict(H=1536, I=8960, KV=256), "7b": dict(H=3584, I=18944, KV=512)}[model]
H, I, KV = SH["H"], SH["I"], SH["KV"]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for group, ns in (("qkv", [H, KV, KV]), ("gate_up", [I, I])):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((T, H), generator=g, device="cuda").to(torch.bfloat16)
    ws = [torch.randn((n, H), generator=g, device="cuda").to(torch.bfloat16) * 0.02 for n in ns]
    dys = [torch.randn((T, n), generator=g, device="cuda").to(torch.bfloat16) for n in ns]
    wf = torch.cat(ws)
    dyf = torch.cat(dys, dim=1).contiguous()
    dx = torch.empty((T, H), device="cuda", dtype=torch.bfloat16)
    gw = [torch.zeros_like(w) for w in ws]
    gwf = torch.zeros_like(wf)
    res = {"model": model, "T": T, "group": group, "N": ns}
    res["fwd_sep_ms"] = timed(lambda: [gemm.linear_fwd(x, w) for w in ws])
    res["fwd_fused_ms"] = timed(lambda: gemm.linear_fwd(x, wf))
    if group == "qkv":  # Qwen2's q/k/v carry a bias: in the GEMM epilogue (prl_gemm) or torch's F.linear
        bs = [torch.randn(n, generator=g, device="cuda").to(torch.bfloat16) for n in ns]
        bf = torch.cat(bs)
        res["fwd_bias_sep_ms"] = timed(lambda: [gemm.linear_fwd(x, w, b) for w, b in zip(ws, bs)])
        res["fwd_bias_sep_torch_ms"] = timed(lambda: [torch.nn.functional.linear(x, w, b) for w, b in zip(ws, bs)])
        res["fwd_bias_fused_ms"] = timed(lambda: gemm.linear_fwd(x, wf, bf))
        res["fwd_bias_fused_torch_ms"] = timed(lambda: torch.nn.functional.linear(x, wf, bf))
        dq = torch.randn((T, ns[0]), generator=g, device="cuda").to(torch.bfloat16)
        res["cat_dy_ms"] = timed(lambda: torch.cat([dq, dys[1], dys[2]], dim=1))
        res["bias_sum_fused_ms"] = timed(lambda: dyf.sum(0, dtype=torch.float32).to(torch.bfloat16))

    def dgrad_sep():
        gemm.linear_dgrad(dys[0], ws[0], out=dx)
        for dy, w in zip(dys[1:], ws[1:]):
            gemm.linear_dgrad(dy, w, out=dx, accumulate=True)

    res["dgrad_sep_ms"] = timed(dgrad_sep)
    res["dgrad_fused_ms"] = timed(lambda: gemm.linear_dgrad(dyf, wf, out=dx))
    res["wgrad_sep_ms"] = timed(lambda: [gemm.linear_wgrad(dy, x, out=o, accumulate=True) for dy, o in zip(dys, gw)])
    res["wgrad_fused_ms"] = timed(lambda: gemm.linear_wgrad(dyf, x, out=gwf, accumulate=True))
    sep = res["fwd_sep_ms"] + res["dgrad_sep_ms"] + res["wgrad_sep_ms"]
    fused = res["fwd_fused_ms"] + res["dgrad_fused_ms"] + res["wgrad_fused_ms"]
    res["total_sep_ms"], res["total_fused_ms"] = round(sep, 4), round(fused, 4)
    res = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}
    print(json.dumps(res), flush=True)
    del x, ws, dys, wf, dyf, dx, gw, gwf
    torch.cuda.empty_cache()

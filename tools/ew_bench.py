"""Element-wise model-op kernels (csrc/model_ops.hip) at trainer shapes: SwiGLU forward / backward
and RMSNorm forward / backward, HIP-event timed, algorithmic TB/s (measurement tool; A/B builds
with PRL_LIB=<variant .so>).

    python tools/ew_bench.py [--tokens 65536] [--inter 8960] [--hidden 1536]
"""

import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402

from pipelinerl_amd import _native  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--inter", type=int, default=8960)
    ap.add_argument("--hidden", type=int, default=1536)
    ap.add_argument("--rows7b", type=int, default=16384)
    a = ap.parse_args()
    lib = _native.load()
    st = torch.cuda.current_stream().cuda_stream
    T, I, H = a.tokens, a.inter, a.hidden
    g = torch.randn((T, I), device="cuda").to(torch.bfloat16)
    u = torch.randn((T, I), device="cuda").to(torch.bfloat16)
    dh = torch.randn((T, I), device="cuda").to(torch.bfloat16)
    h, dg, du = torch.empty_like(g), torch.empty_like(g), torch.empty_like(g)
    n = g.numel()
    out = {"lib": str(_native.LIB_PATH.name), "T": T, "I": I, "H": H}
    ms = timed(lambda: lib.prl_swiglu_forward(g.data_ptr(), u.data_ptr(), h.data_ptr(), n, st))
    out["swiglu_fwd"] = {"ms": round(ms, 4), "TBps": round(6 * n / ms / 1e9, 3)}
    ms = timed(lambda: lib.prl_swiglu_backward(dh.data_ptr(), g.data_ptr(), u.data_ptr(), dg.data_ptr(), du.data_ptr(), n,
                                               st))
    out["swiglu_bwd"] = {"ms": round(ms, 4), "TBps": round(10 * n / ms / 1e9, 3)}
    del g, u, dh, h, dg, du
    from pipelinerl_amd.finetune.model_ops import RMSNormFn

    for rows, hid in ((T, H), (a.rows7b, 3584)):
        x = torch.randn((rows, hid), device="cuda").to(torch.bfloat16).requires_grad_()
        w = torch.ones(hid, device="cuda", dtype=torch.bfloat16).requires_grad_()
        dy = torch.randn((rows, hid), device="cuda").to(torch.bfloat16)
        y = RMSNormFn.apply(x, w, 1e-6)
        ms_f = timed(lambda: RMSNormFn.apply(x.detach(), w.detach(), 1e-6))
        ms_b = timed(lambda: torch.autograd.grad(y, (x, w), dy, retain_graph=True))
        nb = rows * hid * 2
        out[f"rmsnorm_{rows}x{hid}"] = {"fwd_ms": round(ms_f, 4), "fwd_TBps": round(2 * nb / ms_f / 1e9, 3),
                                        "bwd_ms": round(ms_b, 4), "bwd_TBps": round(3 * nb / ms_b / 1e9, 3)}
        # residual add fused into the norm (AddRMSNormFn): fwd reads res + x, writes h + y; bwd
        # reads dy, h, dh, writes dx
        from pipelinerl_amd.finetune.model_ops import AddRMSNormFn

        res = torch.randn((rows, hid), device="cuda").to(torch.bfloat16).requires_grad_()
        dh = torch.randn((rows, hid), device="cuda").to(torch.bfloat16)
        hh, yy = AddRMSNormFn.apply(res, x, w, 1e-6)
        ms_f = timed(lambda: AddRMSNormFn.apply(res.detach(), x.detach(), w.detach(), 1e-6))
        ms_b = timed(lambda: torch.autograd.grad((hh, yy), (x, w), (dh, dy), retain_graph=True))
        out[f"add_rmsnorm_{rows}x{hid}"] = {"fwd_ms": round(ms_f, 4), "fwd_TBps": round(4 * nb / ms_f / 1e9, 3),
                                            "bwd_ms": round(ms_b, 4), "bwd_TBps": round(4 * nb / ms_b / 1e9, 3)}
        del x, w, dy, y, res, dh, hh, yy
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

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
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""The trainer step's linear-layer GEMMs through prl_gemm (ROCm hipBLASLt, include/prl_gemm.h) vs
torch's own matmul (its bundled hipBLASLt), per (pass, T, N, K): time of each, and prl_gemm's
error against an fp32 GEMM of the same bf16 operands (measurement tool, MI355X).

    python tools/gemm_sweep.py --model 1.5b --tokens 65536,16384

Prints one JSON line per problem.
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402

from pipelinerl_amd import gemm  # noqa: E402

SHAPES = {  # (N, K) of q/o, k/v, gate/up, down, lm_head
    "0.5b": dict(qo=(896, 896), kv=(128, 896), gu=(4864, 896), down=(896, 4864), lm_head=(151936, 896)),
    "1.5b": dict(qo=(1536, 1536), kv=(256, 1536), gu=(8960, 1536), down=(1536, 8960), lm_head=(151936, 1536)),
    "7b": dict(qo=(3584, 3584), kv=(512, 3584), gu=(18944, 3584), down=(3584, 18944), lm_head=(152064, 3584)),
}


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
    ap.add_argument("--model", default="1.5b", choices=list(SHAPES))
    ap.add_argument("--tokens", default="65536")
    ap.add_argument("--lm-head-rows", type=int, default=16384, help="label-row lm_head chunk")
    ap.add_argument("--layers", default="qo,kv,gu,down,lm_head")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    print(json.dumps({"prl_gemm_library": gemm.library()}), flush=True)
    for T in [int(t) for t in a.tokens.split(",")]:
        for layer in a.layers.split(","):
            N, K = SHAPES[a.model][layer]
            t = a.lm_head_rows if layer == "lm_head" else T
            g = torch.Generator(device="cuda").manual_seed(1)
            x = torch.randn((t, K), generator=g, device="cuda").to(torch.bfloat16)
            w = torch.randn((N, K), generator=g, device="cuda").to(torch.bfloat16)
            dy = torch.randn((t, N), generator=g, device="cuda").to(torch.bfloat16)
            for pas in a.passes.split(","):
                if pas == "fwd":
                    ours, ref_fn = (lambda: gemm.linear_fwd(x, w)), (lambda: torch.nn.functional.linear(x, w))
                    exact = lambda: x.float() @ w.float().t()  # noqa: E731
                elif pas == "dgrad":
                    ours, ref_fn = (lambda: gemm.linear_dgrad(dy, w)), (lambda: dy @ w)
                    exact = lambda: dy.float() @ w.float()  # noqa: E731
                else:
                    ours, ref_fn = (lambda: gemm.linear_wgrad(dy, x)), (lambda: dy.t() @ x)
                    exact = lambda: dy.float().t() @ x.float()  # noqa: E731
                flops = 2.0 * t * N * K
                ms_ours, ms_torch = timed(ours), timed(ref_fn)
                ref = exact()
                err = float((ours().float() - ref).abs().max() / ref.abs().max())
                terr = float((ref_fn().float() - ref).abs().max() / ref.abs().max())
                del ref
                print(json.dumps({"model": a.model, "layer": layer, "pass": pas, "T": t, "N": N, "K": K,
                                  "prl_ms": round(ms_ours, 4), "torch_ms": round(ms_torch, 4),
                                  "prl_TFLOPs": round(flops / ms_ours / 1e9, 1),
                                  "torch_TFLOPs": round(flops / ms_torch / 1e9, 1),
                                  "speedup": round(ms_torch / ms_ours, 3), "rel_err": err, "torch_rel_err": terr}),
                      flush=True)
            del x, w, dy
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

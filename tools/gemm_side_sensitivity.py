"""How much each of the C3 step's linear-layer GEMMs (Qwen2.5-7B shapes at 12 000 tokens, the
solutions the product routes to through libprl_gemm, and torch's own matmul for the forward) slows
down while workgroups of another queue are resident: alone, beside ONE asleep side workgroup and
beside 16 (an RCCL collective's channels hold CUs this way while it overlaps the step: DESIGN §5).
Measurement only — nothing here changes which solution the product uses.

    python tools/gemm_side_sensitivity.py [--reps 20]

Prints one JSON line per GEMM."""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pipelinerl-swe_amd"))

from pipelinerl_amd import _native  # noqa: E402
from pipelinerl_amd import gemm as prl_gemm  # noqa: E402

T = 12000
SHAPES = {"qo": (3584, 3584), "kv": (512, 3584), "gate_up": (2 * 18944, 3584), "down": (3584, 18944)}


def med_ms(fn, reps: int) -> float:
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.current_stream().synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(0)
    src = torch.empty(1 << 24, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(device=dev)

    def beside(blocks: int, span_s: float):
        """prl_paced_read workgroups that read two 64 KiB turns each and sleep out span_s."""
        nbytes = 2 * blocks * 65536
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            _native.check(lib.prl_paced_read(ctypes.c_void_p(src.data_ptr()), nbytes, nbytes / span_s / 1e9, blocks,
                                             ctypes.c_void_p(sink.data_ptr()), side.cuda_stream), "prl_paced_read")
        torch.cuda._sleep(2_000_000)  # ~1 ms: the side workgroups are resident first

    for name, (N, K) in SHAPES.items():
        x = torch.randn((T, K), generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn((N, K), generator=g, device=dev) * 0.02).to(torch.bfloat16)
        dy = torch.randn((T, N), generator=g, device=dev).to(torch.bfloat16)
        passes = {"fwd": lambda: prl_gemm.linear_fwd(x, w), "dgrad": lambda: prl_gemm.linear_dgrad(dy, w),
                  "wgrad": lambda: prl_gemm.linear_wgrad(dy, x), "torch_fwd": lambda: torch.matmul(x, w.t())}
        for p, fn in passes.items():
            for _ in range(3):
                fn()
            alone = med_ms(fn, a.reps)
            row = {"gemm": name, "N": N, "K": K, "T": T, "pass": p, "alone_ms": round(alone, 4),
                   "routed": prl_gemm.solution_for(p, T, N, K) if p != "torch_fwd" else "torch"}
            span = 3 * a.reps * alone / 1e3 + 0.05
            for blocks in (1, 16):
                beside(blocks, span)
                t = med_ms(fn, a.reps)
                torch.cuda.synchronize()
                row[f"beside_{blocks}wg_ms"] = round(t, 4)
                row[f"ratio_{blocks}wg"] = round(t / alone, 3)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

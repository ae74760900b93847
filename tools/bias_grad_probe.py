"""Bias-gradient reductions (db = dY summed over tokens) on one MI355X: torch's sum(0) with an fp32
accumulator vs a [1, T] x [T, N] GEMM against a ones row (measurement tool)."""
import json
import sys
from pathlib import Path

import torch

sys.path[:0] = [str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd")]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for T, N in ((65536, 1536), (65536, 256), (16384, 3584), (16384, 512)):
    dy = torch.randn((T, N), device="cuda").to(torch.bfloat16)
    ones = torch.ones((1, T), device="cuda", dtype=torch.bfloat16)
    a = dy.sum(0, dtype=torch.float32).to(torch.bfloat16)
    b = (ones @ dy)[0]
    err = float((a.float() - b.float()).abs().max() / a.float().abs().max())
    r = {"T": T, "N": N, "sum_ms": round(timed(lambda: dy.sum(0, dtype=torch.float32).to(torch.bfloat16)), 4),
         "ones_gemm_ms": round(timed(lambda: ones @ dy), 4), "rel_err": err,
         "GBps_at_sum": round(T * N * 2 / timed(lambda: dy.sum(0, dtype=torch.float32)) / 1e6, 1)}
    print(json.dumps(r), flush=True)

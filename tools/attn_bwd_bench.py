"""Time the HIP flash-attention kernels through PackedCausalAttention (tools; rocprofv3 gives the
per-kernel split): forward alone and forward + backward, D 128, GQA native, packed sequences.

    python tools/attn_bwd_bench.py                  # 1.5B (12/2 heads) and 7B (28/4) shapes, 8x2048 and 2x8192
    python tools/attn_bwd_bench.py 16384 2048 12 2  # one configuration: T seq H Hkv

Prints one JSON line per configuration; TFLOP/s counts the causal half of the score matrix
(fwd 4 T seq/2 H D flops, bwd 2.5x that)."""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd.finetune.attention import PackedCausalAttention  # noqa: E402

D = 128


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def run(T, seq, H, HKV, lens=None):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16).requires_grad_()
               for h in (H, HKV, HKV))
    do = torch.randn((T, H, D), generator=g, device="cuda").to(torch.bfloat16)
    bounds = list(range(0, T + 1, seq)) if lens is None else [sum(lens[:i]) for i in range(len(lens) + 1)]
    seq = max(lens) if lens else seq
    cu = torch.tensor(bounds, dtype=torch.int32, device="cuda")

    def fwd():
        with torch.no_grad():
            PackedCausalAttention.apply(q, k, v, cu, seq, bounds)

    def fwd_bwd():
        PackedCausalAttention.apply(q, k, v, cu, seq, bounds).backward(do)

    f_ms, fb_ms = timed(fwd), timed(fwd_bwd)
    flops_f = \
        sum(4.0 * (b - a) * ((b - a) / 2) * H * D for a, b in zip(bounds, bounds[1:]))
    return {"T": T, "seq": seq, "lens": [b - a for a, b in zip(bounds, bounds[1:])], "H": H, "Hkv": HKV,
            "lib": os.environ.get("PRL_LIB", "in-tree"),
            "fwd_ms": round(f_ms, 4), "fwd_TFLOPs": round(flops_f / f_ms / 1e9, 1),
            "fwd_bwd_ms": round(fb_ms, 4), "bwd_ms": round(fb_ms - f_ms, 4),
            "bwd_TFLOPs": round(2.5 * flops_f / (fb_ms - f_ms) / 1e9, 1)}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "lens":  # lens H Hkv l1,l2,...: ragged packing
        H, HKV = int(sys.argv[2]), int(sys.argv[3])
        for spec in sys.argv[4:]:
            lens = [int(x) for x in spec.split(",")]
            print(json.dumps(run(sum(lens), max(lens), H, HKV, lens)), flush=True)
        sys.exit(0)
    if len(sys.argv) > 1:
        cfgs = [tuple(int(x) for x in sys.argv[1:5])]
    else:
        cfgs = [(16384, 2048, 12, 2), (16384, 8192, 12, 2), (16384, 2048, 28, 4), (16384, 8192, 28, 4)]
    for c in cfgs:
        print(json.dumps(run(*c)), flush=True)

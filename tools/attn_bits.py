"""Bit-identity check of the attention backward across two builds (tools; run once per build):

    python tools/attn_bits.py                              # in-tree build
    PRL_LIB=.../variants/libprl_hip_attn_nopipe.so python tools/attn_bits.py

Prints one JSON line per packing with the SHA-256 of dq, dk, dv (bf16 bit patterns) of the HIP
backward (PackedCausalAttention, split plan as the trainer runs it) on fixed random inputs."""
import hashlib
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd.finetune.attention import PackedCausalAttention  # noqa: E402

D = 128
PACKS = [(28, 4, [8511]), (28, 4, [3755, 1617, 6053]), (12, 2, [2048, 2048, 130, 3000]), (40, 8, [1, 700, 2900, 3100])]


def digest(t):
    return hashlib.sha256(t.detach().contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    for H, HKV, lens in PACKS:
        bounds = [sum(lens[:i]) for i in range(len(lens) + 1)]
        T = bounds[-1]
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v = (torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16).requires_grad_()
                   for h in (H, HKV, HKV))
        do = torch.randn((T, H, D), generator=g, device="cuda").to(torch.bfloat16)
        cu = torch.tensor(bounds, dtype=torch.int32, device="cuda")
        out = PackedCausalAttention.apply(q, k, v, cu, max(lens), bounds)
        out.backward(do)
        print(json.dumps({"H": H, "Hkv": HKV, "lens": lens, "out": digest(out), "dq": digest(q.grad),
                          "dk": digest(k.grad), "dv": digest(v.grad)}), flush=True)


if __name__ == "__main__":
    main()

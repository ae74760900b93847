"""Time the attention backward's two workgroup roles apart (tools; no product change): the fused
launch (prl_attn_bwd_split, as the trainer runs it), the same launch with only its dK/dV
workgroups (no query items) and with only its dQ workgroups (no key items, no split units).

    python tools/attn_role_split.py            # C3's packings (workloads.micro_batches("c3")) at 28 / 4 heads
    python tools/attn_role_split.py lens 28 4 8192,8192
    PRL_SPLIT_SWEEP=1.2,0.6,0.3 python tools/attn_role_split.py   # the fused launch per split threshold
    PRL_SPLIT_SWEEP=1.2 PRL_SPLIT_CAPS=1,0.5,0.25 python tools/attn_role_split.py   # per part cap (x target)

Prints one JSON line per packing: ms of each launch and TFLOP/s of the fused one (5 causal
products, 10 L^2/2 H D flops per sequence)."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
from pipelinerl_amd import _native  # noqa: E402
from pipelinerl_amd.finetune import attention  # noqa: E402
from pipelinerl_amd.finetune.attention import BLOCK, _items, _split_items  # noqa: E402

D = 128


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def run(lens, H, HKV, ratio=None, cap=None):
    T = sum(lens)
    bounds = [sum(lens[:i]) for i in range(len(lens) + 1)]
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16) for h in (H, HKV, HKV))
    do = torch.randn((T, H, D), generator=g, device="cuda").to(torch.bfloat16)
    cu = torch.tensor(bounds, dtype=torch.int32, device="cuda")
    lib = _native.load()
    st = torch.cuda.current_stream().cuda_stream
    _, q_items, n = _items(bounds, q.device)
    out = torch.empty_like(q)
    lse2 = torch.empty((H, T), dtype=torch.float32, device="cuda")
    _native.check(lib.prl_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), q_items.data_ptr(), n, out.data_ptr(),
                                   lse2.data_ptr(), T, H, HKV, D, D ** -0.5, st), "prl_attn_fwd")
    delta = torch.empty((H, T), dtype=torch.float32, device="cuda")
    _native.check(lib.prl_attn_bwd_delta(out.data_ptr(), do.data_ptr(), delta.data_ptr(), T, H, D, st), "delta")
    if ratio is not None or cap is not None:  # another split plan (host arithmetic only)
        attention.SPLIT_MIN_RATIO = attention.SPLIT_MIN_RATIO if ratio is None else ratio
        attention.SPLIT_CAP_FRAC = attention.SPLIT_CAP_FRAC if cap is None else cap
        attention._SPLITS.clear()
    kv_s, n_kv, units, n_units, groups, n_groups, slots = _split_items(bounds, H, HKV, q.device)
    parts = torch.empty((max(slots, 1), 2, BLOCK, D), dtype=torch.float32, device="cuda")
    dq, dk, dv = torch.zeros_like(q), torch.zeros_like(k), torch.zeros_like(v)

    def launch(nkv, nq, nu, ng):
        _native.check(lib.prl_attn_bwd_split(
            q.data_ptr(), k.data_ptr(), v.data_ptr(), do.data_ptr(), lse2.data_ptr(), delta.data_ptr(),
            kv_s.data_ptr(), nkv, q_items.data_ptr(), nq, units.data_ptr(), nu, groups.data_ptr(), ng,
            parts.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), T, H, HKV, D, D ** -0.5, st), "bwd")

    full = timed(lambda: launch(n_kv, n, n_units, n_groups))
    dkdv = timed(lambda: launch(n_kv, 0, n_units, n_groups))
    dqo = timed(lambda: launch(0, n, 0, 0))
    fwd = timed(lambda: lib.prl_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), q_items.data_ptr(), n,
                                         out.data_ptr(), lse2.data_ptr(), T, H, HKV, D, D ** -0.5, st))
    area = sum(L * L / 2 for L in lens)
    flops5 = 10 * area * H * D
    return {"lens": lens, "H": H, "Hkv": HKV, "split_min_ratio": attention.SPLIT_MIN_RATIO,
            "split_cap_frac": attention.SPLIT_CAP_FRAC, "fwd_ms": round(fwd, 4), "bwd_ms": round(full, 4),
            "dkdv_only_ms": round(dkdv, 4), "dq_only_ms": round(dqo, 4), "split_units": n_units,
            "bwd_TFLOPs_5prod": round(flops5 / full / 1e9, 1),
            "dkdv_TFLOPs_4prod": round(0.8 * flops5 / dkdv / 1e9, 1),
            "dq_TFLOPs_3prod": round(0.6 * flops5 / dqo / 1e9, 1)}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "lens":
        H, HKV = int(sys.argv[2]), int(sys.argv[3])
        packs = [[int(x) for x in s.split(",")] for s in sys.argv[4:]]
    else:
        import numpy as np

        from pipelinerl_amd import workloads

        H, HKV = 28, 4
        packs = []
        for b in workloads.micro_batches("c3", 4, seed=1234):
            pos = np.asarray(b.position_ids).reshape(-1)
            starts = np.flatnonzero(pos == 0)
            packs.append([int(x) for x in np.diff(np.append(starts, len(pos)))])
    import os

    ratios = [float(x) for x in os.environ.get("PRL_SPLIT_SWEEP", "").split(",") if x] or [None]
    caps = [float(x) for x in os.environ.get("PRL_SPLIT_CAPS", "").split(",") if x] or [None]
    for lens in packs:
        for r in ratios:
            for c in caps:
                print(json.dumps(run(lens, H, HKV, r, c)), flush=True)


if __name__ == "__main__":
    main()

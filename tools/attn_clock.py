"""In-kernel clock and MFMA-pipe occupancy of the attention backward (diagnostic build only).

    python tools/build_variants.py attn_clock     # here: PRL_ATTN_CLOCK_PROBE=1 build
    PRL_LIB=pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_attn_clock.so python tools/attn_clock.py
    ... python tools/attn_clock.py lens 28 4 8192,8192

The probe build stamps (s_memtime, s_memrealtime) at the start and end of every workgroup of
attn_bwd_fused (wave 0) into a buffer nothing else reads.  After >= 2 s of back-to-back launches
(MI355X_MICROARCH.md, DVFS item 6) one more launch is read back: per workgroup the shader clock =
d(memtime) / d(realtime) x 100 MHz, and its MFMA-pipe occupancy = (the MFMAs its busiest wave
issues x 32 cycles) / d(memtime) (dK/dV: 32 per live 32-query tile per query head, wave 0;
dQ: 24 per live 32-key tile, wave 3), and wave 0's cycles split by phase of the stage loop
(barrier wait, LDS stage store + barrier, issuing the next stage's loads, paired tiles, single
masked tiles).  Prints one JSON line per packing.
"""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
from pipelinerl_amd import _native  # noqa: E402
from pipelinerl_amd.finetune.attention import BLOCK, _items, _split_items  # noqa: E402

D = 128


def run(lens, H, HKV):
    T = sum(lens)
    bounds = [sum(lens[:i]) for i in range(len(lens) + 1)]
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16) for h in (H, HKV, HKV))
    do = torch.randn((T, H, D), generator=g, device="cuda").to(torch.bfloat16)
    lib = _native.load()
    clock_read = getattr(lib, "prl_attn_clock_read", None)
    if clock_read is None:
        raise SystemExit("not a PRL_ATTN_CLOCK_PROBE build (set PRL_LIB to variants/libprl_hip_attn_clock.so)")
    clock_read.restype, clock_read.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]
    st = torch.cuda.current_stream().cuda_stream
    _, q_items, n = _items(bounds, q.device)
    out = torch.empty_like(q)
    lse2 = torch.empty((H, T), dtype=torch.float32, device="cuda")
    _native.check(lib.prl_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), q_items.data_ptr(), n, out.data_ptr(),
                                   lse2.data_ptr(), T, H, HKV, D, D ** -0.5, st), "prl_attn_fwd")
    delta = torch.empty((H, T), dtype=torch.float32, device="cuda")
    _native.check(lib.prl_attn_bwd_delta(out.data_ptr(), do.data_ptr(), delta.data_ptr(), T, H, D, st), "delta")
    kv_s, n_kv, units, n_units, groups, n_groups, slots = _split_items(bounds, H, HKV, q.device)
    parts = torch.empty((max(slots, 1), 2, BLOCK, D), dtype=torch.float32, device="cuda")
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)

    def launch():
        _native.check(lib.prl_attn_bwd_split(
            q.data_ptr(), k.data_ptr(), v.data_ptr(), do.data_ptr(), lse2.data_ptr(), delta.data_ptr(),
            kv_s.data_ptr(), n_kv, q_items.data_ptr(), n, units.data_ptr(), n_units, groups.data_ptr(), n_groups,
            parts.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), T, H, HKV, D, D ** -0.5, st), "bwd")

    t_end = time.perf_counter() + 2.0
    reps = 0
    while time.perf_counter() < t_end:
        for _ in range(10):
            launch()
        torch.cuda.synchronize()
        reps += 10
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    launch()
    e.record()
    torch.cuda.synchronize()
    wall_ms = s.elapsed_time(e)
    grid = n_units + n_kv * HKV + n * H
    buf = (ctypes.c_ulonglong * (4 * grid))()
    _native.check(clock_read(ctypes.addressof(buf), grid), "prl_attn_clock_read")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(grid, 4).astype(np.float64)
    cyc, real = a[:, 2] - a[:, 0], (a[:, 3] - a[:, 1]) * 10.0  # ns
    phase_read = lib.prl_attn_phase_read
    phase_read.restype, phase_read.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]
    pbuf = (ctypes.c_ulonglong * (8 * grid))()
    _native.check(phase_read(ctypes.addressof(pbuf), grid), "prl_attn_phase_read")
    ph = np.frombuffer(pbuf, dtype=np.uint64).reshape(grid, 8).astype(np.float64)
    ghz = cyc / np.maximum(real, 1.0)
    pair_read = getattr(lib, "prl_attn_pair_read", None)
    pair = None
    if pair_read is not None:
        pair_read.restype, pair_read.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]
        qbuf = (ctypes.c_ulonglong * (8 * grid))()
        _native.check(pair_read(ctypes.addressof(qbuf), grid), "prl_attn_pair_read")
        pair = np.frombuffer(qbuf, dtype=np.uint64).reshape(grid, 8).astype(np.float64)

    # MFMAs of each workgroup's busiest wave, in launch order
    u = units.cpu().numpy().reshape(-1, 7)[:n_units] if n_units else np.zeros((0, 7), np.int64)
    kvr = kv_s.cpu().numpy().reshape(-1, 3)[:n_kv]
    mf = [32 * (r[5] - r[4]) * -(-(r[1] - r[2]) // 32) for r in u]
    mf += [32 * (H // HKV) * -(-(r[1] - r[2]) // 32) for r in kvr for _ in range(HKV)]
    n_kv_wg = len(mf)
    qr = q_items.cpu().numpy().reshape(-1, 3)[:n]
    mf += [24 * -(-(min(r[2] + BLOCK, r[1]) - r[0]) // 32) for r in qr for _ in range(H)]  # per role: order-free sums
    mf = np.asarray(mf, np.float64)
    kv, qq = slice(0, n_kv_wg), slice(n_kv_wg, grid)
    area = sum(L * L / 2 for L in lens)
    extra = {}
    if pair is not None:
        # wave 0's cycles per region of the pair schedule, per pair: each region issues 16 MFMAs
        # (dQ: 16, 16, 8, 8), so 512 / 512 / 256 / 256 cycles would be the MFMA-bound floor
        names = {"dkdv": ("S_a_dP_a", "S_b_dP_b+softmax_a", "acc_a+softmax_b", "acc_b"),
                 "dq": ("S_a_dP_a", "S_b_dP_b+softmax_a", "acc_a+softmax_b", "acc_b")}
        extra["pair_region_cycles"] = {
            role: {nm: round(float(pair[sl, i].sum() / max(pair[sl, 4].sum(), 1.0)), 1) for i, nm in enumerate(names[role])}
            for role, sl in (("dkdv", kv), ("dq", qq))}
        extra["pairs_per_wg"] = {role: round(float(pair[sl, 4].mean()), 1) for role, sl in (("dkdv", kv), ("dq", qq))}
    return {**extra,"lens": lens, "H": H, "Hkv": HKV, "workgroups": grid, "warm_launches": reps, "wall_ms": round(wall_ms, 4),
            "clock_ghz": {"median": round(float(np.median(ghz)), 3), "p10": round(float(np.percentile(ghz, 10)), 3),
                          "p90": round(float(np.percentile(ghz, 90)), 3)},
            "mfma_pipe_busy": {"dkdv": round(float(32 * mf[kv].sum() / cyc[kv].sum()), 3),
                               "dq": round(float(32 * mf[qq].sum() / cyc[qq].sum()), 3)},
            "wg_us_mean": {"dkdv": round(float(real[kv].mean() / 1e3), 1), "dq": round(float(real[qq].mean() / 1e3), 1)},
            # wave 0's shader cycles by phase of the stage loop, as fractions of the workgroups' cycles
            # (dK/dV: wave 0 has the most tiles; dQ: the fewest, so its barrier share includes waiting for wave 3)
            "wave0_phase_frac": {role: {name: round(float(ph[sl, i].sum() / cyc[sl].sum()), 3) for i, name in
                                        enumerate(("barrier_wait", "stage_store_and_barrier", "load_issue",
                                                   "paired_tiles", "single_tiles"))}
                                 for role, sl in (("dkdv", kv), ("dq", qq))},
            "stages_per_wg": {"dkdv": round(float(ph[kv, 5].mean()), 1), "dq": round(float(ph[qq, 5].mean()), 1)},
            "bwd_TFLOPs_5prod": round(10 * area * H * D / wall_ms / 1e9, 1),
            "peak_TFLOPs_at_median_clock": round(2.5e3 * float(np.median(ghz)) / 2.4, 1)}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "lens":
        H, HKV = int(sys.argv[2]), int(sys.argv[3])
        packs = [[int(x) for x in s.split(",")] for s in sys.argv[4:]]
    else:
        from pipelinerl_amd import workloads

        H, HKV = 28, 4
        packs = []
        for b in workloads.micro_batches("c3", 4, seed=1234):
            pos = np.asarray(b.position_ids).reshape(-1)
            starts = np.flatnonzero(pos == 0)
            packs.append([int(x) for x in np.diff(np.append(starts, len(pos)))])
    for lens in packs:
        print(json.dumps(run(lens, H, HKV)), flush=True)


if __name__ == "__main__":
    os.environ.setdefault("PRL_ATTN_SPLIT", "1")
    main()

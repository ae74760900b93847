"""Calibrate FETCH_SIZE for the fp32 loss head's access pattern (round 6).

The gfx950 correction in MI355X_MICROARCH.md (FETCH_SIZE x 2 for 16-B/lane streaming reads) puts
the bf16 resident kernel at 1.005x its algorithmic bytes but both fp32 kernels at ~1.115x, all
reads (WRITE_SIZE matches the dlogits bytes).  The guide says other patterns are uncalibrated, so
this runs, in one process and in a fixed order, kernels whose read bytes are known:

  copy39   prl_paced_read over the 39.8 GB fp32 logits tensor (T = 65536, V = 151 936), 1024 WGs
  copy20   prl_paced_read over its first half (19.9 GB)
  pair_T   the fp32 loss head (pair kernel) at T = 65536, V = 151 936 (39.8 GB of logits)
  pair_h   the same at T = 32768 (19.9 GB: the footprint halved, rows unchanged)
  pair_v   T = 65536, V = 75 968 (19.9 GB: rows halved, grpo_fwd_pair_f32<10>)

``--reps`` launches each.  Under ``rocprofv3 --pmc FETCH_SIZE`` (and a separate WRITE_SIZE pass)
``--summarize FETCH_DIR WRITE_DIR`` groups the dispatches by kernel and order, and prints each
arm's corrected bytes over its known bytes.
"""

from __future__ import annotations

import argparse
import csv
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

V0, T0 = 151936, 65536
ARMS = [("copy39", None), ("copy20", None), ("pair_T", (T0, V0)), ("pair_h", (T0 // 2, V0)),
        ("pair_v", (T0, V0 // 2))]


def run(reps: int) -> None:
    import torch

    import bench
    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    dev = torch.device("cuda", 0)
    lib = _native.load()
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    buf = torch.empty(T0 * V0 * 4, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for name, nbytes in (("copy39", buf.numel()), ("copy20", buf.numel() // 2)):
        for _ in range(reps):
            _native.check(lib.prl_paced_read(ctypes.c_void_p(buf.data_ptr()), nbytes, 1.0e6, 1024,
                                             ctypes.c_void_p(sink.data_ptr()), s), "prl_paced_read")
        torch.cuda.synchronize()
        print(json.dumps({"arm": name, "bytes": nbytes, "launches": reps}), flush=True)
    del buf
    torch.cuda.empty_cache()
    for name, (T, V) in ARMS[2:]:
        lb, fields = bench.make_workload(T, V, seq=2048, prompt=256, seed=4321, device=dev)
        logits = lb.detach().float().requires_grad_(True)
        del lb
        for _ in range(reps):
            logits.grad = None
            loss, stats, _ = grpo_loss(logits, fields, params)
            loss.backward()
        torch.cuda.synchronize()
        print(json.dumps({"arm": name, "T": T, "V": V, "read_bytes": T * V * 4, "launches": reps}), flush=True)
        del logits, fields, loss, stats
        torch.cuda.empty_cache()


def _dispatches(d: Path, counter: str) -> list[tuple[int, str, float]]:
    f = next(d.rglob("*counter_collection.csv"))
    per: dict[int, list] = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"]
            if r["Counter_Name"] == counter and ("paced_read" in k or "pair_f32" in k):
                e = per.setdefault(int(r["Dispatch_Id"]), [k, 0.0])
                e[1] += float(r["Counter_Value"])
    return [(i, k, v) for i, (k, v) in sorted(per.items())]


def summarize(fetch_dir: str, write_dir: str, reps: int) -> dict:
    import statistics

    out = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x1024 x2, "
                     "WRITE_SIZE x1024 (MI355X_MICROARCH.md HBM section)", "arms": {}}
    for counter, d in (("FETCH_SIZE", fetch_dir), ("WRITE_SIZE", write_dir)):
        rows = _dispatches(Path(d), counter)
        paced = [v for _, k, v in rows if "paced_read" in k]
        pair = [v for _, k, v in rows if "pair_f32" in k]
        groups = {"copy39": paced[:reps], "copy20": paced[reps:2 * reps],
                  "pair_T": pair[:reps], "pair_h": pair[reps:2 * reps], "pair_v": pair[2 * reps:3 * reps]}
        for name, vals in groups.items():
            if not vals:
                continue
            kb = statistics.median(vals)
            out["arms"].setdefault(name, {})[counter] = kb * 1024 * (2 if counter == "FETCH_SIZE" else 1)
    known = {"copy39": (T0 * V0 * 4, 0), "copy20": (T0 * V0 * 2, 0), "pair_T": (T0 * V0 * 4, T0 * V0 * 4),
             "pair_h": (T0 // 2 * V0 * 4, T0 // 2 * V0 * 4), "pair_v": (T0 * (V0 // 2) * 4, T0 * (V0 // 2) * 4)}
    for name, a in out["arms"].items():
        rd, wr = known[name]
        a["read_known"], a["write_known"] = rd, wr
        if "FETCH_SIZE" in a:
            a["read_over_known"] = round(a["FETCH_SIZE"] / rd, 4)
        if "WRITE_SIZE" in a and wr:
            a["write_over_known"] = round(a["WRITE_SIZE"] / wr, 4)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--summarize", nargs=2, default=None, metavar=("FETCH_DIR", "WRITE_DIR"))
    a = ap.parse_args()
    if a.summarize:
        print(json.dumps(summarize(*a.summarize, a.reps), indent=1))
    else:
        run(a.reps)

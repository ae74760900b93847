"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, csv output) of
bench.py into the per-launch HBM traffic JSON that bench.py's roofline reads.

  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json
  python tools/pmc_traffic.py --fp32 gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r05_fp32_pmc.json
      (the bench's loss_head_fp32 probe: every fp32 loss-head kernel found, per-launch medians)

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section, gfx950): FETCH_SIZE is in
KB and counts 16-B/lane streaming reads at half rate (x1024 x2); WRITE_SIZE is in KB (x1024).
"""

from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

KERNEL = "grpo_fwd_resident<19>"
T, V = 65536, 151936


def per_launch(d: Path, counter: str) -> tuple[float, int]:
    f = next(d.rglob("*counter_collection.csv"))
    vals: dict[str, float] = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {f}")
    lo, hi = min(vals.values()), max(vals.values())
    if hi > 1.1 * lo:  # the same kernel at another shape (e.g. the label-row path) was traced too
        raise SystemExit(f"{counter}: launches of {KERNEL} differ ({lo:.0f} .. {hi:.0f} KB): not all at T={T}")
    return sum(vals.values()) / len(vals), len(vals)


def main(fetch_dir: str, write_dir: str, out: str) -> None:
    fkb, n = per_launch(Path(fetch_dir), "FETCH_SIZE")
    wkb, _ = per_launch(Path(write_dir), "WRITE_SIZE")
    rd, wr = fkb * 1024 * 2, wkb * 1024
    alg = 2.0 * T * V * 2 + T * 37
    res = {"kernel": f"prl::{KERNEL}", "T": T, "V": V, "dtype": "bf16",
           "FETCH_SIZE_KB_per_launch": fkb, "WRITE_SIZE_KB_per_launch": wkb,
           "read_bytes_corrected": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
           "algorithmic_bytes": alg, "traffic_over_algorithmic": (rd + wr) / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, --output-format csv, "
                     "bench.py --steps 3 --warmup 1 --no-cpu-baseline; FETCH_SIZE x1024 x2 (gfx950 half-count on "
                     "16-B/lane streaming reads), WRITE_SIZE x1024; mean over launches",
           "launches": n}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


def fp32_main(fetch_dir: str, write_dir: str, out: str) -> None:
    """Per-launch medians of every fp32 loss-head kernel the two passes traced (pair / hybrid)."""
    import statistics

    def rows(d: Path, counter: str) -> dict[str, list[float]]:
        f = next(d.rglob("*counter_collection.csv"))
        per: dict[tuple[str, str], float] = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if ("pair_f32" in k or "hybrid_f32" in k) and r["Counter_Name"] == counter:
                    key = (k, r["Dispatch_Id"])
                    per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        out: dict[str, list[float]] = {}
        for (k, _), v in per.items():
            out.setdefault(k, []).append(v)
        return out

    fetch, write = rows(Path(fetch_dir), "FETCH_SIZE"), rows(Path(write_dir), "WRITE_SIZE")
    alg = 2.0 * T * V * 4 + T * 37
    res = {"tool": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of bench.py's loss_head_fp32 probe; "
                   "FETCH_SIZE x 1024 x 2, WRITE_SIZE x 1024 (MI355X_MICROARCH.md HBM section)",
           "T": T, "V": V, "per_launch_median": {}}
    for k in sorted(set(fetch) & set(write)):
        rd = statistics.median(fetch[k]) * 1024 * 2
        wr = statistics.median(write[k]) * 1024
        res["per_launch_median"][k] = {"fetch_size_bytes": rd, "write_size_bytes": wr, "algorithmic_bytes": alg,
                                       "traffic_over_algorithmic": round((rd + wr) / alg, 4),
                                       "launches": [len(fetch[k]), len(write[k])]}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


def adamw_main(fetch_dir: str, write_dir: str, out: str, params: str = "7615616512") -> None:
    """prl_adamw_master_step over a model (tools/adamw_master_bench.py): HBM bytes per optimizer step
    (all adamw_master_kernel dispatches of a pass / the steps it ran; 11 launches per 7B step) against
    28 algorithmic bytes per parameter.  FETCH_SIZE x1024 x2 (the guide's gfx950 correction for 16-B
    per-lane streaming reads: the fp32 master / moment loads; the bf16 gradient loads are 8 B per lane,
    uncalibrated — read_bytes_uncorrected is given beside), WRITE_SIZE x1024."""
    def total(d: Path, counter: str) -> tuple[float, int]:
        f = next(d.rglob("*counter_collection.csv"))
        per: dict[str, float] = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "adamw_master_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        return sum(per.values()), len(per)

    fkb, nf = total(Path(fetch_dir), "FETCH_SIZE")
    wkb, nw = total(Path(write_dir), "WRITE_SIZE")
    n = int(params)
    steps_f, steps_w = nf / 11, nw / 11
    rd, wr = fkb * 1024 * 2 / steps_f, wkb * 1024 / steps_w
    alg = 28.0 * n
    res = {"kernel": "prl::adamw_master_kernel (prl_adamw_master_step)", "params": n, "launches_per_step": 11,
           "steps": [steps_f, steps_w], "read_bytes_per_step": rd, "read_bytes_uncorrected": fkb * 1024 / steps_f,
           "write_bytes_per_step": wr, "bytes_per_step": rd + wr, "algorithmic_bytes": alg,
           "traffic_over_algorithmic": round((rd + wr) / alg, 4),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, --output-format csv, "
                     "tools/adamw_master_bench.py --model 7b --steps 2"}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "--fp32":
        fp32_main(*sys.argv[2:5])
    elif sys.argv[1] == "--adamw":
        adamw_main(*sys.argv[2:5])
    else:
        main(*sys.argv[1:4])

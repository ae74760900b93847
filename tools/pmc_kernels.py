"""Fold rocprofv3 PMC passes (csv output, one directory per pass) into a per-kernel table:
mean counter value per dispatch, for every kernel whose name contains one of the given
substrings.

  python tools/pmc_kernels.py out.json attn_fwd,attn_bwd_fused gpurun_out/pmc_a gpurun_out/pmc_b ...

Derived fractions (when the counters are present; SQ_* cycle counters of the SQ block count
quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES and SQ_BUSY_CU_CYCLES, MI355X_MICROARCH.md constants table):
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked at s_waitcnt / barrier)
  stall_frac  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls: MFMA RAW, pipe busy, LDS issue)
  active_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
"""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def fold(dirs: list[Path], keys: list[str]) -> dict:
    acc: dict[str, dict[str, dict[str, float]]] = defaultdict(lambda: defaultdict(dict))
    for d in dirs:
        for f in d.rglob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"]
                    k = next((k for k in keys if k in name), None)
                    if k is None:
                        continue
                    per = acc[k][r["Counter_Name"]]
                    per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    out = {}
    for k, counters in acc.items():
        row = {c: sum(v.values()) / len(v) for c, v in counters.items()}
        row["dispatches"] = max(len(v) for v in counters.values())
        w = row.get("SQ_WAVE_CYCLES")
        if w:
            for num, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "stall_frac"),
                              ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if num in row:
                    row[name] = round(row[num] / w, 4)
        out[k] = row
    return out


if __name__ == "__main__":
    res = fold([Path(p) for p in sys.argv[3:]], sys.argv[2].split(","))
    Path(sys.argv[1]).write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))

"""PMC summary of the packed-attention kernels (VERDICT r05 item 6's evidence): per kernel, the
per-dispatch mean of each SQ counter over two rocprofv3 --pmc passes of tools/attn_bwd_bench.py,
and the fractions read from them:

  wait_frac    SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waves waiting on anything)
  active_frac  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (waves issuing)
  mfma_util    SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES)

    bash tools/attn_pmc.sh            # the two passes -> gpurun_out/attn_pmc1, attn_pmc2
    python tools/attn_pmc.py gpurun_out/attn_pmc1 gpurun_out/attn_pmc2 > profiles/r06_attention_pmc.json
"""
import csv
import json
import sys
from pathlib import Path

KERNELS = ("attn_fwd", "attn_bwd_fused", "attn_bwd_delta", "attn_bwd_dkdv_reduce")


def per_kernel(d: Path) -> dict:
    out: dict = {}
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
                if name is None:
                    continue
                disp = out.setdefault(name, {}).setdefault(r["Dispatch_Id"], {})
                disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main(*dirs: str) -> dict:
    res: dict = {}
    for d in dirs:
        for k, disps in per_kernel(Path(d)).items():
            acc = res.setdefault(k, {})
            for counters in disps.values():
                for c, v in counters.items():
                    acc.setdefault(c, []).append(v)
    out = {}
    for k, acc in res.items():
        m = {c: sum(v) / len(v) for c, v in acc.items()}
        m["dispatches"] = max(len(v) for v in acc.values())
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_WAIT_ANY" in m:
                m["wait_frac"] = round(m["SQ_WAIT_ANY"] / wc, 4)
            if "SQ_ACTIVE_INST_ANY" in m:
                m["active_frac"] = round(m["SQ_ACTIVE_INST_ANY"] / wc, 4)
        if m.get("SQ_BUSY_CU_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            m["mfma_util"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_BUSY_CU_CYCLES"]), 4)
        out[k] = m
    return out


if __name__ == "__main__":
    print(json.dumps(main(*sys.argv[1:]), indent=1))

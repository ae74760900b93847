"""Merge tools/hipblaslt_probe.bin sweep lines (JSONL) into pipelinerl_amd/gemm_solutions.json:
for each problem whose fastest solution beats the library heuristic by > 3 %, record
{T, index, ms, heuristic_ms} under "pass:N:K:dtype:accumulate" ("wgrad32" = the fp32 accumulating
lm_head weight gradient, "wgradacc" = a bf16 weight gradient added into .grad, beta = 1).  prl_gemm uses an entry for token counts within 2x of its T.

    python tools/gemm_solutions_from_sweep.py profiles/r01_hipblaslt_rocm72_sweep_*.jsonl
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "pipelinerl-swe_amd" / "pipelinerl_amd" / "gemm_solutions.json"


def main(paths):
    table = json.loads(OUT.read_text()) if OUT.exists() else {}
    n = 0
    for p in paths:
        for line in Path(p).read_text().splitlines():
            d = json.loads(line)
            if not d.get("best") or d["heuristic_ms"] <= 0 or d["best"][0]["ms"] >= 0.97 * d["heuristic_ms"]:
                continue
            pas, f32, acc = {"wgrad32": ("wgrad", True, True), "wgradacc": ("wgrad", False, True)}.get(
                d["pass"], (d["pass"], False, False))
            key = f"{pas}:{d['N']}:{d['K']}:{'f32' if f32 else 'bf16'}:{int(acc)}"
            ent = [e for e in table.get(key, []) if e["T"] != d["T"]]
            ent.append({"T": d["T"], "index": d["best"][0]["index"], "ms": d["best"][0]["ms"],
                        "heuristic_ms": d["heuristic_ms"]})
            table[key] = sorted(ent, key=lambda e: e["T"])
            n += 1
    OUT.write_text(json.dumps(table, indent=1, sort_keys=True) + "\n")
    print(f"{n} entries merged into {OUT} ({len(table)} problems)")


if __name__ == "__main__":
    main(sys.argv[1:])

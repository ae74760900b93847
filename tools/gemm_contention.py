"""How much longer the step's kernels run while a side-stream kernel holds a few CUs, from a
rocprofv3 kernel trace (tools/c3_step.py --snapshot --paced-arms ... under --kernel-trace).

    python tools/gemm_contention.py <kernel_trace.csv> [--side paced_read] [--out summary.json]

For every dispatch NOT matching ``--side``: whether it overlapped a ``--side`` dispatch in time.
Per kernel name seen both ways: median duration inside vs outside the side kernel's windows; per
class (gemm / attention / other, step_flops.kernel_class): the summed extra time, i.e. what the
side kernel cost the step beside it."""

from __future__ import annotations

import argparse
import bisect
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tools")]

from kernel_overlap import load, merged  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--side", default="paced_read")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from pipelinerl_amd.step_flops import kernel_class

    rows = load(a.trace)
    side = merged([(t0, t1) for t0, t1, n, _ in rows if a.side in n])
    starts = [s for s, _ in side]

    def overlaps(t0, t1):
        i = bisect.bisect_right(starts, t1) - 1
        while i >= 0 and side[i][1] >= t0:
            if side[i][0] <= t1:
                return True
            i -= 1
        return False

    inside: dict[str, list[int]] = {}
    outside: dict[str, list[int]] = {}
    for t0, t1, n, _ in rows:
        if a.side in n:
            continue
        (inside if overlaps(t0, t1) else outside).setdefault(n, []).append(t1 - t0)
    per, by_class = [], {}
    for n, d_in in inside.items():
        d_out = outside.get(n)
        if not d_out or len(d_out) < 3:
            continue
        m_in, m_out = statistics.median(d_in), statistics.median(d_out)
        extra = sum(d_in) - m_out * len(d_in)
        c = kernel_class(n)
        by_class.setdefault(c, {"extra_ms": 0.0, "inside_ms": 0.0, "dispatches_inside": 0})
        by_class[c]["extra_ms"] += extra / 1e6
        by_class[c]["inside_ms"] += sum(d_in) / 1e6
        by_class[c]["dispatches_inside"] += len(d_in)
        per.append({"kernel": n[:120], "class": c, "n_inside": len(d_in), "n_outside": len(d_out),
                    "median_inside_us": round(m_in / 1e3, 1), "median_outside_us": round(m_out / 1e3, 1),
                    "ratio": round(m_in / m_out, 3), "extra_ms": round(extra / 1e6, 3)})
    per.sort(key=lambda r: -r["extra_ms"])
    res = {"side_kernel": a.side, "side_windows_ms": round(sum(b - s for s, b in side) / 1e6, 2),
           "by_class": {k: {kk: round(vv, 3) if isinstance(vv, float) else vv for kk, vv in v.items()}
                        for k, v in by_class.items()},
           "top": per[:25]}
    txt = json.dumps(res, indent=1)
    if a.out:
        Path(a.out).write_text(txt)
    print(txt)


if __name__ == "__main__":
    main()

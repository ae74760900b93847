"""How much of one kernel's time other kernels ran beside it, from a rocprofv3 kernel trace.

    python tools/kernel_overlap.py <kernel_trace.csv> <name regex> [--skip-first-calls N] [--out summary.json]

For every dispatch whose Kernel_Name matches the regex: its duration and the part of it during which
at least one dispatch NOT matching the regex was running (any queue).  Used for the weight-update
snapshot (prl_flatten_bf16 on WeightUpdateManager's side stream) against the C3 step's kernels:
``overlapped_frac`` near 1 means the snapshot ran concurrently with the trainer's next step rather
than serialised with it (tools/c3_step.py --snapshot under rocprofv3 --kernel-trace).  Dispatches
less than 50 us apart form one call (a snapshot is one flatten call = one dispatch per 32 tensors);
``--skip-first-calls 4`` leaves out the probe's snapshot-alone timing, which runs first.  Each
timed arm ends with a device synchronize, so the last snapshot of an arm has no next step beside
it: the per-call list shows which calls had one."""

from __future__ import annotations

import argparse
import bisect
import csv
import json
import re


def load(path: str) -> list[tuple[int, int, str, str]]:
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            t0 = int(r.get("Start_Timestamp") or r.get("BeginNs") or 0)
            t1 = int(r.get("End_Timestamp") or r.get("EndNs") or 0)
            q = r.get("Queue_Id") or r.get("Stream_Id") or ""
            if t1 > t0:
                rows.append((t0, t1, name, q))
    return rows


def merged(intervals: list[tuple[int, int]]) -> list[tuple[int, int]]:
    out: list[list[int]] = []
    for a, b in sorted(intervals):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


def covered(a: int, b: int, spans: list[tuple[int, int]], starts: list[int]) -> int:
    """Length of [a, b) covered by the disjoint sorted spans."""
    i = max(0, bisect.bisect_right(starts, a) - 1)
    tot = 0
    while i < len(spans) and spans[i][0] < b:
        lo, hi = max(a, spans[i][0]), min(b, spans[i][1])
        if hi > lo:
            tot += hi - lo
        i += 1
    return tot


def summarize(rows, pattern: str, skip_first_calls: int = 0, gap_ns: int = 50_000) -> dict:
    rx = re.compile(pattern)
    mine = sorted((a, b, q) for a, b, n, q in rows if rx.search(n))
    calls: list[list[tuple[int, int, str]]] = []
    for d in mine:
        if calls and d[0] - calls[-1][-1][1] <= gap_ns:
            calls[-1].append(d)
        else:
            calls.append([d])
    skipped = calls[:skip_first_calls]
    calls = calls[skip_first_calls:]
    mine = [d for c in calls for d in c]
    others = merged([(a, b) for a, b, n, _ in rows if not rx.search(n)])
    starts = [a for a, _ in others]
    per = []
    for a, b, q in mine:
        per.append({"start_ns": a, "dur_us": round((b - a) / 1e3, 2), "queue": q,
                    "overlapped_us": round(covered(a, b, others, starts) / 1e3, 2)})
    dur = sum(p["dur_us"] for p in per)
    ov = sum(p["overlapped_us"] for p in per)
    per_call, i = [], 0
    for c in calls:
        seg = per[i:i + len(c)]
        i += len(c)
        cd, co = sum(p["dur_us"] for p in seg), sum(p["overlapped_us"] for p in seg)
        per_call.append({"start_ns": seg[0]["start_ns"], "dispatches": len(seg), "dur_us": round(cd, 1),
                         "overlapped_us": round(co, 1), "overlapped_frac": round(co / cd, 4) if cd else None})
    return {"kernel": pattern, "dispatches": len(per), "calls": len(per_call),
            "skipped_first_calls": [{"dispatches": len(c), "dur_us": round(sum(b - a for a, b, _ in c) / 1e3, 1)}
                                    for c in skipped],
            "per_call": per_call, "total_us": round(dur, 1), "overlapped_us": round(ov, 1),
            "overlapped_frac": round(ov / dur, 4) if dur else None,
            "queues": sorted({p["queue"] for p in per}),
            "other_kernel_queues": sorted({q for a, b, n, q in rows if not rx.search(n)}),
            "per_dispatch": per[:64]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pattern")
    ap.add_argument("--skip-first-calls", type=int, default=0)
    ap.add_argument("--out")
    a = ap.parse_args()
    s = summarize(load(a.trace), a.pattern, a.skip_first_calls)
    text = json.dumps(s, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(json.dumps({k: v for k, v in s.items() if k not in ("per_dispatch", "per_call")}))


if __name__ == "__main__":
    main()

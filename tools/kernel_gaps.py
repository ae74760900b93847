"""GPU idle gaps from a rocprofv3 --kernel-trace CSV (measurement tool): total kernel-busy time vs
the span, and the largest gaps with the kernels around them.

    python tools/kernel_gaps.py <kernel_trace.csv> [min_gap_us] [top]
"""
import csv
import sys
from collections import Counter

f = sys.argv[1]
min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
busy, end, gaps = 0, rows[0][0], []
for i, (a, b, n) in enumerate(rows):
    if a > end:
        gaps.append((a - end, i))
    busy += max(0, b - max(a, end))
    end = max(end, b)
span = end - rows[0][0]
print(f"kernels {len(rows)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {(span - busy) / 1e6:.1f} ms")
big = [(g, i) for g, i in gaps if g >= min_gap * 1e3]
print(f"gaps >= {min_gap} us: {len(big)}, total {sum(g for g, _ in big) / 1e6:.1f} ms")
by_prev = Counter()
for g, i in big:
    by_prev[rows[i - 1][2][:60]] += g
for n, g in by_prev.most_common(10):
    print(f"  after {n}: {g / 1e6:.1f} ms")
for g, i in sorted(big, reverse=True)[:top]:
    print(f"{g / 1e3:9.1f} us  after {rows[i - 1][2][:50]}  before {rows[i][2][:50]}")

"""Gaps between consecutive kernels of the last greedy-decode call in a rocprofv3 --kernel-trace CSV
(tools/prof_decode.py under rocprofv3 --kernel-trace --output-format csv): wall span, kernel-busy time, the
gap histogram, and per kernel name the mean duration and mean gap in front of it.

Usage: python tools/decode_gaps.py <kernel_trace.csv>"""

import csv
import sys
from collections import defaultdict


def main(path: str):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[1])
    cuts = [i for i in range(1, len(rows)) if rows[i][1] - rows[i - 1][2] > 1_000_000]
    call = rows[cuts[-1]:] if cuts else rows
    span = call[-1][2] - call[0][1]
    busy = sum(e - s for _, s, e in call)
    print(f"kernels {len(call)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
    hist = defaultdict(lambda: [0, 0])
    per = defaultdict(lambda: [0, 0, 0])
    for i in range(1, len(call)):
        g = call[i][1] - call[i - 1][2]
        b = "<0" if g < 0 else "<1us" if g < 1000 else "1-2us" if g < 2000 else "2-5us" if g < 5000 else ">5us"
        hist[b][0] += 1
        hist[b][1] += g
        k = call[i][0].split("(")[0][:90]
        per[k][0] += 1
        per[k][1] += call[i][2] - call[i][1]
        per[k][2] += g
    for b in ("<0", "<1us", "1-2us", "2-5us", ">5us"):
        if b in hist:
            print(f"  gaps {b:6s} n={hist[b][0]:5d} total {hist[b][1] / 1e6:.3f} ms")
    print(f"{'n':>6} {'avg_us':>8} {'gap_us':>8}  kernel")
    for k, (n, d, g) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"{n:6d} {d / n / 1e3:8.2f} {g / n / 1e3:8.2f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])

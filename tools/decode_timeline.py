"""Timeline of the last greedy-decode call in a rocprofv3 kernel-trace database (tools/prof_decode.py under
rocprofv3 --kernel-trace): wall span, kernel-busy time, idle gaps between consecutive kernels (launch floor, host
sync between graph chunks), and the largest gaps with the kernels either side.

Usage: python tools/decode_timeline.py <results.db> [kernels_per_call]"""

import sqlite3
import sys


def main(db: str, per_call: int = 0):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if per_call <= 0:  # split calls at gaps > 1 ms (the host's synchronize between generate calls)
        cuts = [i for i in range(1, len(rows)) if rows[i][1] - rows[i - 1][2] > 1_000_000]
        start = cuts[-1] if cuts else 0
    else:
        start = len(rows) - per_call
    call = rows[start:]
    span = call[-1][2] - call[0][1]
    busy = sum(e - s for _, s, e in call)
    gaps = [(call[i][1] - call[i - 1][2], i) for i in range(1, len(call))]
    print(f"kernels {len(call)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
    hist = {}
    for g, _ in gaps:
        b = "<1us" if g < 1000 else "1-2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">20us"
        hist[b] = hist.get(b, [0, 0])
        hist[b][0] += 1
        hist[b][1] += g
    for b in ("<1us", "1-2us", "2-5us", "5-20us", ">20us"):
        if b in hist:
            print(f"  gaps {b:7s} n={hist[b][0]:5d} total {hist[b][1] / 1e6:.3f} ms")
    for g, i in sorted(gaps, reverse=True)[:8]:
        print(f"  gap {g / 1e3:8.1f} us  after {call[i - 1][0][:70]}  before {call[i][0][:70]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)

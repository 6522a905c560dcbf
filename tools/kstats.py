"""Summarise a rocprofv3 results database (kernel trace) into a per-kernel table (for profiles/).

    python tools/kstats.py run_results.db "title"                       # every kernel of the traced run
    python tools/kstats.py run_results.db "title" --window adam_update_kernel 3 8

--window MARK SKIP COUNT restricts the table to the kernels that ran after the SKIP-th launch whose name contains
MARK ended and up to the end of the (SKIP + COUNT)-th one: with the optimizer kernel as MARK, exactly COUNT train
steps (the bench's timed graph replays after its warm-up steps), and the table gains a per-step column."""

import sqlite3
import sys


def main(db: str, title: str = "", window=None):
    c = sqlite3.connect(db)
    where, per = "", None
    if window:
        mark, skip, count = window[0], int(window[1]), int(window[2])
        ends = [r[0] for r in c.execute("select end from kernels where name like ? order by start", (f"%{mark}%",))]
        if len(ends) < skip + count:
            raise SystemExit(f"kstats: {len(ends)} launches of {mark}, window needs {skip + count}")
        lo = ends[skip - 1] if skip > 0 else 0
        hi = ends[skip + count - 1]
        where = f" where start > {lo} and end <= {hi}"
        per = count
        span = (hi - lo) / 1e6
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) from kernels"
                     + where + " group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = [title]
    if per:
        out.append(f"window: {per} steps, span {span:.3f} ms ({span / per:.3f} ms/step), kernel busy {tot / 1e6:.3f} ms "
                   f"({tot / 1e6 / per:.3f} ms/step)")
    out.append(f"{'total_ms':>9} {'pct':>5} {'calls':>6} " + (f"{'/step':>6} " if per else "") +
               f"{'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel")
    for r in rows:
        out.append(f"{r[2] / 1e6:9.3f} {100 * r[2] / tot:5.1f} {r[1]:6d} " + (f"{r[1] / per:6.1f} " if per else "") +
                   f"{r[3] / 1e3:9.2f} {r[4] / 1e3:9.2f} {r[5] / 1e3:9.2f}  {r[0][:150]}")
    print("\n".join(out))


if __name__ == "__main__":
    a = sys.argv[1:]
    w = None
    if "--window" in a:
        i = a.index("--window")
        w = a[i + 1:i + 4]
        a = a[:i] + a[i + 4:]
    main(a[0], a[1] if len(a) > 1 else "", w)

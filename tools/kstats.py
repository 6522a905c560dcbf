"""Summarise a rocprofv3 results database (kernel trace) into a per-kernel table (for profiles/)."""

import sqlite3
import sys


def main(db: str, title: str = ""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = [title, f"{'total_ms':>9} {'pct':>5} {'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel"]
    for r in rows:
        out.append(f"{r[2] / 1e6:9.3f} {100 * r[2] / tot:5.1f} {r[1]:6d} {r[3] / 1e3:9.2f} {r[4] / 1e3:9.2f} "
                   f"{r[5] / 1e3:9.2f}  {r[0][:150]}")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")

"""Per-kernel PMC totals (summed over instances per dispatch, averaged over dispatches) from a rocprofv3 .db."""

import sqlite3
import sys


def main(db: str, like: str = "%"):
    c = sqlite3.connect(db)
    q = ("select name, counter_name, sum(counter_value), count(distinct dispatch_id), avg(duration) from pmc_events "
         "where name like ? group by name, counter_name order by name, counter_name")
    cur = None
    for name, cn, tot, nd, dur in c.execute(q, (like,)):
        if name != cur:
            print(f"{name[:110]}  (dispatches {nd}, avg {dur / 1e3:.1f} us)")
            cur = name
        print(f"    {cn:28s} {tot / nd:16.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "%")

"""Per-launch SQ counters of the plain 8320x2304x768 GEMM, before / after the r02 epilogue change
(tools/k768_probe.sh output): prints one table for profiles/."""
import glob
import sqlite3
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/k768"
res = {}
for lib in ("before", "current"):
    for tag in ("a", "b"):
        for db in glob.glob(f"{root}/{tag}_{lib}/*.db"):
            c = sqlite3.connect(db)
            q = ("select name, counter_name, sum(counter_value), count(distinct dispatch_id) from pmc_events "
                 "where name like '%gemm_kernel%' group by name, counter_name")
            for name, cn, tot, nd in c.execute(q):
                res.setdefault(lib, {})[cn] = tot / nd
                res[lib]["kernel"] = name[:70]
names = sorted({k for d in res.values() for k in d if k != "kernel"})
print(f"{'counter (per launch)':28s} {'before':>16s} {'current':>16s} {'ratio':>7s}")
for n in names:
    b, a = res.get("before", {}).get(n), res.get("current", {}).get(n)
    r = f"{a / b:7.3f}" if a and b else ""
    print(f"{n:28s} {b if b is not None else float('nan'):16.0f} {a if a is not None else float('nan'):16.0f} {r}")
for lib, d in res.items():
    print(lib, d.get("kernel"))

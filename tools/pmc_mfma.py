"""Per-kernel MFMA utilisation from a rocprofv3 PMC .db (tools/pmc_mfma.sh).

util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs): the fraction of SIMD-cycles
with a matrix op in flight while the kernel ran (GRBM_GUI_ACTIVE is summed over the 8 XCDs). A bf16
16x16x32 MFMA holds its SIMD 16 cycles for 16384 flops, so busy cycles x 1024 = MFMA flops executed (tile
padding included) — per launch it is what bench.py's roofline divides by the launch time (the dominant GEMM: 36.5
GF/launch here vs 36.5 algorithmic). Durations under --pmc are inflated by the profiler's serialisation, so
utilisation uses the counted GRBM cycles, not the wall time."""

import sqlite3
import sys


def main(db: str):
    c = sqlite3.connect(db)
    q = ("select name, counter_name, sum(counter_value), count(distinct dispatch_id), sum(duration) "
         "from pmc_events group by name, counter_name")
    agg = {}
    for name, cn, tot, nd, _ in c.execute(q):
        agg.setdefault(name, {})[cn] = (tot, nd)
    durs = {n: (d, k) for n, d, k in c.execute(
        "select name, sum(duration), count(distinct dispatch_id) from pmc_events "
        "where counter_name = 'GRBM_GUI_ACTIVE' group by name")}
    rows = []
    for name, d in agg.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        busy, nd = d["SQ_VALU_MFMA_BUSY_CYCLES"]
        grbm, _ = d["GRBM_GUI_ACTIVE"]
        dur_ns, _ = durs.get(name, (0, nd))
        util = busy / (grbm / 8.0 * 256 * 4) if grbm else 0.0
        gf = busy * 1024.0 / max(nd, 1) / 1e9
        kcyc = grbm / 8.0 / max(nd, 1) / 1e3
        rows.append((kcyc, util, gf, nd, grbm, name))
    rows.sort(key=lambda r: -r[4])
    tot = sum(r[4] for r in rows)
    w_util = sum(r[1] * r[4] for r in rows) / tot if tot else 0.0
    print("# rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE over bench.py --steps 2 "
          "--warmup 1 --no-graph --no-decode (4 eager train steps incl. warm-ups)")
    print(f"# cycle-weighted MFMA util over all kernels of the step: {w_util:.3f}")
    print(f"{'kcyc/launch':>11} {'mfma_util':>9} {'mfma_GF/launch':>14} {'calls':>5}  kernel")
    for kcyc, util, gf, nd, _, name in rows[:40]:
        print(f"{kcyc:11.1f} {util:9.3f} {gf:14.3f} {nd:5d}  {name[:120]}")


if __name__ == "__main__":
    main(sys.argv[1])

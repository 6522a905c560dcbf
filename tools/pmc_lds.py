"""Per-kernel LDS counters from a rocprofv3 PMC .db (tools/pmc_lds.sh): SQ_LDS_BANK_CONFLICT (extra cycles),
SQ_LDS_IDX_ACTIVE (all LDS-array cycles), SQ_LDS_UNALIGNED_STALL, summed over each kernel's dispatches; conflict
share = BANK_CONFLICT / IDX_ACTIVE (MI355X_MICROARCH.md: the fraction of LDS cycles spent on bank conflicts)."""

import sqlite3
import sys

CN = ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_UNALIGNED_STALL")


def main(db: str):
    c = sqlite3.connect(db)
    agg = {}
    for name, cn, tot, nd in c.execute("select name, counter_name, sum(counter_value), count(distinct dispatch_id) "
                                       "from pmc_events group by name, counter_name"):
        agg.setdefault(name, {})[cn] = (tot, nd)
    rows = []
    for name, d in agg.items():
        if CN[1] not in d:
            continue
        idx, nd = d[CN[1]]
        bc = d.get(CN[0], (0, nd))[0]
        us = d.get(CN[2], (0, nd))[0]
        rows.append((idx, name, nd, bc, us))
    rows.sort(reverse=True)
    print(f"{'launches':>8} {'LDS_IDX_ACTIVE/launch':>22} {'BANK_CONFLICT/launch':>21} {'conflict share':>14} "
          f"{'UNALIGNED/launch':>16}  kernel")
    for idx, name, nd, bc, us in rows[:40]:
        print(f"{nd:8d} {idx / nd:22.0f} {bc / nd:21.0f} {bc / max(idx, 1):14.3f} {us / nd:16.0f}  {name[:140]}")


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel (JSON for
profiles/; bench.py reports the entry of its dominant kernel as roofline.traffic).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over XCD instances here). On gfx950 FETCH_SIZE tallies
wide (16 B/lane) reads at half their bytes (MI355X_MICROARCH.md, HBM): bytes = 2 x FETCH + WRITE. The copy probe
(1 GiB read + 1 GiB write) is reported beside it as the calibration.

usage: pmc_traffic.py FETCH_DB WRITE_DB OUT_JSON [calib_fetch_db calib_write_db]"""

import json
import sqlite3
import sys


def per_dispatch(db, counter):
    c = sqlite3.connect(db)
    q = ("select name, sum(counter_value), count(distinct dispatch_id) from pmc_events where counter_name = ? "
         "group by name")
    return {n: (v / d, d) for n, v, d in c.execute(q, (counter,))}


def short(name):
    i = name.find("(")
    n = name[:i] if i > 0 else name
    return n[5:] if n.startswith("void ") else n


def main():
    fdb, wdb, out = sys.argv[1:4]
    f, w = per_dispatch(fdb, "FETCH_SIZE"), per_dispatch(wdb, "WRITE_SIZE")
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
    for name, (fk, n) in sorted(f.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        wk = w.get(name, (0.0, 0))[0]
        res["kernels"][short(name)] = {"dispatches": n, "fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
                                       "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024))}
    if len(sys.argv) > 5:
        cf, cw = per_dispatch(sys.argv[4], "FETCH_SIZE"), per_dispatch(sys.argv[5], "WRITE_SIZE")
        k = max(cf, key=lambda n: cf[n][0])
        res["calibration"] = {"kernel": short(k)[:80], "bytes_read": 1 << 30, "bytes_written": 1 << 30,
                              "fetch_kib": round(cf[k][0], 1), "write_kib": round(cw.get(k, (0, 0))[0], 1)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()

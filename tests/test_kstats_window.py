"""tools/kstats.py --window: the per-step kernel table the profiles/ kstats files are made from counts exactly the
kernels between the end of the SKIP-th optimizer launch and the end of the (SKIP + COUNT)-th (CPU: a synthetic
rocprofv3-shaped database)."""

import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kstats  # noqa: E402


def _db(path, steps):
    c = sqlite3.connect(path)
    c.execute("create table kernels (name text, start integer, end integer, duration integer)")
    t = 0
    c.execute("insert into kernels values (?, ?, ?, ?)", ("build_fold_gemm", t, t + 500, 500))
    t += 1000
    for _ in range(steps):
        for name, d in (("gemm_kernel<A>", 300), ("gemm_kernel<A>", 300), ("ln_bwd8_kernel", 100),
                        ("adam_update_kernel", 200)):
            c.execute("insert into kernels values (?, ?, ?, ?)", (name, t, t + d, d))
            t += d + 10
    c.commit()
    c.close()


def test_window_counts_the_timed_steps(tmp_path, capsys):
    db = str(tmp_path / "run_results.db")
    _db(db, 12)
    kstats.main(db, "t", ["adam_update_kernel", "3", "8"])
    out = capsys.readouterr().out.splitlines()
    assert out[1].startswith("window: 8 steps")
    rows = {ln.split()[-1]: ln.split() for ln in out[3:]}
    assert "build_fold_gemm" not in rows  # the one-time build launch is outside the window
    assert rows["gemm_kernel<A>"][2] == "16" and rows["gemm_kernel<A>"][3] == "2.0"  # calls, calls per step
    assert rows["adam_update_kernel"][2] == "8" and rows["ln_bwd8_kernel"][2] == "8"


def test_whole_run_without_window(tmp_path, capsys):
    db = str(tmp_path / "run_results.db")
    _db(db, 12)
    kstats.main(db, "t")
    out = capsys.readouterr().out.splitlines()
    rows = {ln.split()[-1]: ln.split() for ln in out[2:]}
    assert rows["gemm_kernel<A>"][2] == "24" and rows["build_fold_gemm"][2] == "1"

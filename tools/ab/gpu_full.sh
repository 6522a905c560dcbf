#!/bin/bash
# full GPU test suite, then the short bench with per-shape GEMM timings, then the kernel-time table
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/full; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
ICAP_GEMM_DETAIL=$O/gemm_detail.txt timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-decode --sweep "" > $O/bench.json 2> $O/bench.err
rc=$?; tail -1 $O/bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "packed bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -24 $O/kstats.txt | cut -c1-150
rm -rf $O/p

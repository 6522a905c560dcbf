#!/bin/bash
# Round-2 closing pass (one gpurun call): every -m gpu test, the configs[4] bench line, the kernel-time profile of the
# headline train step, then the default bench line. Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/round2; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large.json 2> $O/bench_large.err || exit $?
tail -1 $O/bench_large.json | cut -c1-300
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -12 $O/kstats.txt | cut -c1-150
rm -rf $O/p
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-300; exit $rc

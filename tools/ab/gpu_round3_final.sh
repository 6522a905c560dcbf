#!/bin/bash
# round-3 pass: every -m gpu test, the default bench line, the kernel-time table and PMC traffic of the step,
# then the configs[4] lines (fp8 + bf16). Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/r3f; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -1 $O/bench.json | cut -c1-300; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "packed bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -12 $O/kstats.txt | cut -c1-150
rm -rf $O/p
bash tools/pmc_traffic.sh r3f/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
timeout -k 10 600 python -u bench.py --config large --fp8 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large_fp8.json 2> $O/bench_large_fp8.err || exit $?
tail -1 $O/bench_large_fp8.json | cut -c1-250
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline --no-decode > $O/bench_large_bf16.json 2> $O/bench_large_bf16.err || exit $?
tail -1 $O/bench_large_bf16.json | cut -c1-250

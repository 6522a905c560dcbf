#!/bin/bash
# Closing pass: epilogue-activation probe, every -m gpu test, kernel-time profile of the headline step, the default
# bench line and the configs[4] line. Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/final; mkdir -p $O; cd $R
timeout -k 10 120 python -u tools/act_epilogue_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/act_probe.txt || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -10 $O/kstats.txt | cut -c1-150
rm -rf $O/p
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large.json 2> $O/bench_large.err; rc=$?
tail -1 $O/bench_large.json | cut -c1-200; exit $rc

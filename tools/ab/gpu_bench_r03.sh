#!/bin/bash
# Round-3 bench pass: default bench line (with the batch sweep), configs[4] fp8 and bf16 lines.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/r03b; mkdir -p $O; cd $R
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config large --fp8 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large_fp8.json 2> $O/bench_large_fp8.err || exit $?
tail -1 $O/bench_large_fp8.json | cut -c1-300
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline --no-decode > $O/bench_large_bf16.json 2> $O/bench_large_bf16.err || exit $?
tail -1 $O/bench_large_bf16.json | cut -c1-300

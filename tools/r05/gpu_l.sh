#!/bin/bash
# bf16 LN race forensics (rounding classification), then the full GPU suite, the bench line and its kernel trace
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
PROBE_BF16=1 timeout -k 10 300 python -u tools/ab/ln_race_f32.py 2>&1 | grep -v amdgpu.ids > $O/ln_bf16.txt; tail -25 $O/ln_bf16.txt
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_lnfold_gpu.py -k greedy 2>&1 | grep -E "agreement|passed|failed" 
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv"

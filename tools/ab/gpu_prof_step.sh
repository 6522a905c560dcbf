#!/bin/bash
# kernel-time breakdown of the bench train step (rocprofv3 kernel trace) + the default bench line
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/prof; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -32 $O/kstats.txt | cut -c1-170
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-400; exit $rc

#!/bin/bash
# kernel-time table of the packed headline step (rocprofv3) + the per-shape GEMM timings of one eager step
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/prof4; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
ICAP_GEMM_DETAIL=$O/gemm_detail.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "packed bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -40 $O/kstats.txt | cut -c1-170
rm -rf $O/p
head -60 $O/gemm_detail.txt | cut -c1-170

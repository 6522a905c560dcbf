#!/bin/bash
# Round-3 profiles: K=768 counter probe, then rocprofv3 kernel-time tables of the headline step and the configs[4]
# fp8 step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/prof3; mkdir -p $O
cd $R && ./tools/k768_probe.sh > $O/k768.log 2>&1; tail -4 $O/k768.log
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "bench train step x (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats.txt && head -14 $O/kstats.txt | cut -c1-150
rm -rf $O/p; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/q -o run -- python3 $R/bench.py --config large --fp8 --steps 4 --warmup 2 --no-decode --no-cpu-baseline > $O/prof_large_fp8.json 2> $O/prof_large.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof_large.err; exit $rc; }
cd $R && python tools/kstats.py $O/q/run_results.db "configs[4] fp8 train step x (2 warm-up + 4 timed + 1 eager roofline pass)" > $O/kstats_large_fp8.txt && head -14 $O/kstats_large_fp8.txt | cut -c1-150
rm -rf $O/q

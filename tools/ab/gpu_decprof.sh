#!/bin/bash
# greedy decode kernel trace (rocprofv3 --kernel-trace, csv) -> per-kernel durations and launch gaps
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/decprof; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/prof_decode.py > $O/prof.log 2>&1; rc=$?
tail -3 $O/prof.log; [ $rc -eq 0 ] || exit $rc
f=$(find $O/trace -name "*kernel_trace.csv" | head -1); python3 $R/tools/decode_gaps.py $f > $O/gaps.txt; rc=$?
cat $O/gaps.txt | head -40; rm -rf $O/trace; exit $rc

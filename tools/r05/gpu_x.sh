#!/bin/bash
# greedy decode: the timed loop, then its kernel trace
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 300 python -u tools/prof_decode.py 2>&1 | grep -v amdgpu.ids | tee $O/decode.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/prof_decode.py > $O/prof_decode.txt 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*.db"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/blt -o run -- python3 -u tools/ab/blaslt_names.py > $O/blaslt.txt 2>&1 || exit 1

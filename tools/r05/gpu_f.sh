#!/bin/bash
# round-5 closing measurements: the bench line, its kernel trace (graph-replay window), HBM traffic by PMC
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['gpt2_block'], d['greedy_captions_per_s'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*.db"
bash tools/pmc_traffic.sh r05f/pmc || exit 1

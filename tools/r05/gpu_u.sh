#!/bin/bash
# full GPU suite, patch-embed timing, the bench line, and its kernel trace (graph-replay window)
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u tools/ab/patch_bench.py 2>&1 | grep -v amdgpu.ids | tee $O/patch_bench.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['gpt2_block'], r.get('replay_roofline'), d['greedy_captions_per_s'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*.db" | head -2
timeout -k 10 600 python -u bench.py --config large --fp8 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_large_fp8.json 2> $O/bench_large_fp8.err || { tail -20 $O/bench_large_fp8.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_large_fp8.json')); print('large fp8', d['value'], d['ms_per_step'], d['roofline']['frac'])"

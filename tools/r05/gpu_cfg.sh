#!/bin/bash
# configs[3] (medium) and configs[4] (large, fp8) bench lines on the final tree
set -o pipefail
O=gpurun_out/r05cfg; mkdir -p $O
timeout -k 10 600 python -u bench.py --config medium --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_medium.json 2> $O/bench_medium.err || { tail -20 $O/bench_medium.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_medium.json')); print('medium', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('greedy_captions_per_s'))"
timeout -k 10 600 python -u bench.py --config large --fp8 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_large_fp8.json 2> $O/bench_large_fp8.err || { tail -20 $O/bench_large_fp8.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_large_fp8.json')); print('large fp8', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('greedy_captions_per_s'))"

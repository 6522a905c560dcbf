#!/bin/bash
# (experiment) K-skew A/B over the whole packed step: ICAP_KSKEW = 0..4, per-shape GEMM tables (eager pass)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/kskew; mkdir -p $O; cd $R
for s in 0 1 2 3 4 0 2; do
  ICAP_GEMM_DETAIL=$O/detail_$s.txt ICAP_KSKEW=$s timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/bench_$s.json 2> $O/bench_$s.err || exit 1
  python -c "import json,sys; d=json.loads(open('$O/bench_$s.json').read().strip().splitlines()[-1]); print('KSKEW=$s', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_ms_per_step'])"
done

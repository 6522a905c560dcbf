#!/bin/bash
# gelu_new-specialised epilogue on the 3-block (variant 4, no spills) vs the 4-block (variant 5) short-K kernel
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/heavy; mkdir -p $O; cd $R
for v in 5 4 5 4; do
  ICAP_VAR_HEAVY=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('heavy=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_ms_per_step'])"
done

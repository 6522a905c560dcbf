#!/bin/bash
# whole-step A/B over the GEMM planner's A/B switches (packed train step, 20 timed steps each)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/envab; mkdir -p $O; cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/b_$tag.json 2> $O/b_$tag.err || return 1
  python -c "import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_ms_per_step'])"
}
for rep in 1 2; do
  run base ICAP_X=0 || exit 1
  run S2 ICAP_FUSED_S=2 || exit 1
  run S3 ICAP_FUSED_S=3 || exit 1
  run S4 ICAP_FUSED_S=4 || exit 1
  run ring ICAP_FUSED_SPLIT_K=0 || exit 1
  run nst1 ICAP_FUSED_NST=1 || exit 1
done

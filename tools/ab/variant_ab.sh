#!/bin/bash
# short-K tile-variant A/B (ICAP_VAR_HEAVY / ICAP_VAR_ACT / ICAP_VAR_LIGHT) over the packed train step
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/varab; mkdir -p $O; cd $R
run() {
  local tag=$1; shift
  env ICAP_GEMM_DETAIL=$O/detail_$tag.txt "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/b_$tag.json 2> $O/b_$tag.err || return 1
  python -c "import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_ms_per_step'])"
}
run base ICAP_X=0 || exit 1
run H4 ICAP_VAR_HEAVY=4 || exit 1
run H0 ICAP_VAR_HEAVY=0 || exit 1
run A0 ICAP_VAR_ACT=0 || exit 1
run A5 ICAP_VAR_ACT=5 || exit 1
run L0 ICAP_VAR_LIGHT=0 || exit 1
run L5 ICAP_VAR_LIGHT=5 || exit 1
run base2 ICAP_X=0 || exit 1

#!/bin/bash
# Interleaved A/B of the headline train step under environment switches (same box, same process image):
#   tools/ab/train_ab.sh OUTDIR "NAME=ENV[,ENV...]" ...   e.g. tools/ab/train_ab.sh gpurun_out/ab "fold1=" "fold0=ICAP_TRAIN_LN_FOLD=0"
# (several switches in one form are comma-separated: "adam=ICAP_ADAM_U=2,ICAP_ADAM_NT=1")
# Each form runs bench.py's headline only (no decode / CPU baseline / sweep / unfrozen line), twice, interleaved.
set -o pipefail
O=$1; shift; mkdir -p $O
for rep in 1 2; do
  for form in "$@"; do
    name=${form%%=*}; envs=${form#*=}; envs=${envs//,/ }
    env $envs timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-decode --no-cpu-baseline --sweep "" --no-unfrozen > $O/$name.$rep.json 2> $O/$name.$rep.err || { tail -3 $O/$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'rep', sys.argv[3], d['value'], 'images/s', d['ms_per_step_median'], 'ms median', 'eager', d['roofline'].get('eager_step_ms'))" $O/$name.$rep.json $name $rep
  done
done

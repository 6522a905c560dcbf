#!/bin/bash
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
export PROBE_VICTIMS=ln_bwd_bare,ln_bwd PROBE_AGGRESSORS=none,tile,kout PROBE_REPS=8
echo "== no packed-fp32 (VOP3P v_pk_*_f32) in layernorm.hip: -fno-slp-vectorize" > $O/matrix.txt
ICAP_LIB=tools/ab/_libs/libicap_nopk.so timeout -k 10 300 python -u tools/ab/ln_race_probe.py 2>&1 | grep -v amdgpu.ids | grep -v "fit:" >> $O/matrix.txt; rc=$?
cat $O/matrix.txt; exit $rc

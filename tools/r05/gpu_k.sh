#!/bin/bash
# LN backward side-stream victim: mean/rstd load order variants (ICAP_LIB = diagnostic builds of layernorm.hip)
set -o pipefail
mkdir -p gpurun_out/r05k
export PROBE_VICTIMS=ln_bwd_bare,ln_bwd PROBE_AGGRESSORS=none,tile,kout
run() {  # name, then env assignments
  local n=$1; shift
  echo "== $n" | tee -a gpurun_out/r05k/matrix.txt
  env "$@" timeout -k 10 300 python -u tools/ab/ln_race_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05k/matrix.txt
}
run "original order (mean/rstd first)" ICAP_LIB=tools/ab/_libs/libicap_ln0.so && \
run "original order + const mean" ICAP_LIB=tools/ab/_libs/libicap_ln0.so PROBE_CONST_MEAN=1 && \
run "mean/rstd first + vmcnt(0)" ICAP_LIB=tools/ab/_libs/libicap_ln1.so && \
run "product (mean/rstd with the chunk loads)" PROBE_X=1

#!/bin/bash
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "attn or attention or mapper or parity or greedy or decode or beam" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for L in old new; do
  lib=""; [ $L = old ] && lib=$PWD/tools/ab/_libs/libicap_attn_old.so
  echo "== $L" | tee -a $O/attn_bench.txt
  ICAP_LIB=$lib timeout -k 10 200 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids | tee -a $O/attn_bench.txt
done
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 200 python -u tools/ab/lmhead_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/lmhead.txt

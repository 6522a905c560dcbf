#!/bin/bash
# in-launch split-K A/B on the packed N=768 products: split count and main-loop variant
mkdir -p gpurun_out
for cfg in "ICAP_FUSED_S=0" "ICAP_FUSED_S=2" "ICAP_FUSED_S=3" "ICAP_FUSED_S=4" "ICAP_FUSED_S=6" "ICAP_FUSED_NST=2" "ICAP_FUSED_NST=2 ICAP_FUSED_S=2" "ICAP_FUSED_SPLIT_K=0"; do
  echo "== $cfg"
  env $cfg timeout -k 5 120 python3 tools/gemm_live_bench.py 2>&1 | grep -E "768x 3072|768x 2304"
done

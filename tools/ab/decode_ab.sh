#!/bin/bash
# greedy decode (B=128 x 50) with the shipped library vs A/B builds (ICAP_LIB), alternating rounds
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/decab; mkdir -p $O; cd $R
for i in 1 2; do
  timeout -k 10 120 python -u tools/prof_decode.py 2>&1 | grep decode | sed 's/^/shipped: /' || exit 1
  for LIB in "$@"; do
    ICAP_LIB=$R/$LIB timeout -k 10 120 python -u tools/prof_decode.py 2>&1 | grep decode | sed "s#^#$LIB: #" || exit 1
  done
done

#!/bin/bash
# attention A/B: tools/ab_cur (the build before the change) vs the current build, interleaved, twice each
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/ab_attn; mkdir -p $O; cd $R
for i in 1 2; do
  ICAP_LIB=$R/tools/ab_cur/libicap_hip.so timeout -k 10 60 python3 tools/attn_bench.py 2>&1 | sed 's/^/before /' | tee -a $O/ab.txt || exit 1
  timeout -k 10 60 python3 tools/attn_bench.py 2>&1 | sed 's/^/after  /' | tee -a $O/ab.txt || exit 1
done
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q -k "attn or attention or train or graph" --timeout 120 --timeout-method thread 2>&1 | tail -2

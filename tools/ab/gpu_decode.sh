#!/bin/bash
# Decode work: per-launch microbench, then the GPU tests that run the skinny GEMMs / decode path.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/dec; mkdir -p $O; cd $R
timeout -k 10 200 python -u tools/decode_bench.py > $O/bench.txt 2>&1; rc=$?; cat $O/bench.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_parity_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|bf16 |passed|failed" $O/pytest.log | tail -15; exit $rc

#!/bin/bash
# 256x256 GEMM: correctness tests first (bounded), then the per-shape timing table
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/g256; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py > $O/gemm_bench.txt 2>&1; rc=$?; cat $O/gemm_bench.txt | grep -v amdgpu.ids; exit $rc

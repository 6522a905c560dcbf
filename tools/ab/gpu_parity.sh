#!/bin/bash
# Parity tests of the round-2 goldens + the ring GEMM tests (one GPU call)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); mkdir -p $R/gpurun_out/parity; cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -v -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/parity/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|bf16 greedy|passed|failed" gpurun_out/parity/pytest.log | tail -40
exit $rc

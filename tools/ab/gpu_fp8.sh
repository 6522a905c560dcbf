#!/bin/bash
# MX fp8: the lane-map probe (host check runs on the CPU afterwards), then the fp8 kernel tests.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/fp8; mkdir -p $O; cd $R
timeout -k 10 60 ./tools/microbench/mx_probe $O/mx_probe.bin || exit $?
python tools/mx_probe_check.py $O/mx_probe.bin > $O/mx_probe_check.txt 2>&1; head -3 $O/mx_probe_check.txt
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py $PYTEST_K -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|assert|fp8 large" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fp8_gemm_bench.py > $O/fp8_gemm_bench.txt 2>&1; rc=$?; cat $O/fp8_gemm_bench.txt; exit $rc

#!/bin/bash
# Round-3 GPU pass: the new tests first (RCCL world-1, two-stream split-K, fused-LN offset, beam layout), then every
# -m gpu test, then the default bench line. Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/r03; mkdir -p $O; cd $R
if [ -x tools/microbench/mx_probe ]; then timeout -k 10 60 ./tools/microbench/mx_probe $O/mx_probe.bin || exit $?; fi
timeout -k 10 400 python -u -m pytest tests/test_dp_nccl_gpu.py tests/test_splitk_streams_gpu.py tests/test_determinism_gpu.py tests/test_beam.py "tests/test_kernels_gpu.py::test_gemm_fused_layernorm_large_mean" -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|offset" $O/pytest_new.log | tail -12; [ $rc -eq 0 ] || exit $rc
if [ "$1" == "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-400; exit $rc
fi

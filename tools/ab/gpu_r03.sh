#!/bin/bash
# Round-3 GPU pass: the new tests first, then (full) every -m gpu test, the default bench line (with the batch sweep)
# and the configs[4] fp8 / bf16 bench lines. Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/r03; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_dp_nccl_gpu.py tests/test_splitk_streams_gpu.py tests/test_determinism_gpu.py tests/test_beam.py tests/test_fp8_gpu.py tests/test_bench_shape_gpu.py "tests/test_kernels_gpu.py::test_gemm_fused_layernorm_large_mean" -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|offset|fp8 large|bench128" $O/pytest_new.log | tail -12; [ $rc -eq 0 ] || exit $rc
if [ "$1" == "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 500 python -u bench.py --config large --fp8 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large_fp8.json 2> $O/bench_large_fp8.err || exit $?
  tail -1 $O/bench_large_fp8.json | cut -c1-300
  timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline --no-decode > $O/bench_large_bf16.json 2> $O/bench_large_bf16.err || exit $?
  tail -1 $O/bench_large_bf16.json | cut -c1-300
fi

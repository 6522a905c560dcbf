#!/bin/bash
# packed-row GEMM microbench + pack tests + short bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_live_bench.py > gpurun_out/live_gemm.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_pack_gpu.py tests/test_bench_shape_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/live_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-decode --sweep "" > gpurun_out/live_bench.log 2>&1
rc=$?
cat gpurun_out/live_gemm.log | grep -v amdgpu.ids
tail -3 gpurun_out/live_tests.log
tail -c 1500 gpurun_out/live_bench.log
exit $rc

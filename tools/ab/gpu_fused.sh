#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_fused_splitk_gpu.py tests/test_splitk_streams_gpu.py tests/test_pack_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_live_bench.py > gpurun_out/fused_gemm.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_bench_shape_gpu.py tests/test_parity_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/fused_tests2.log 2>&1 &&
ICAP_GEMM_DETAIL=gpurun_out/fused_gemm_detail.txt timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-decode --sweep "" > gpurun_out/fused_bench.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/fused_tests.log | tail -30
grep -v amdgpu.ids gpurun_out/fused_gemm.log
tail -3 gpurun_out/fused_tests2.log
tail -c 800 gpurun_out/fused_bench.log
exit $rc

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_live_bench.py > gpurun_out/live_gemm2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/live_gemm2.log; exit $rc

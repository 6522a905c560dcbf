#!/bin/bash
# 192 x 64 tiles on the LDS-DMA ring for long K: bitwise tests, then the per-shape A/B
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w192_gpu.py 2>&1 | tail -15 | tee $O/test.txt || exit 1
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 300 python -u tools/ab/w192_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.txt

#!/bin/bash
# variant 24 (192 x 64 tiles): its bitwise tests, then the A/B against the automatic plan and hipBLASLt
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w192_gpu.py 2>&1 | tail -15 | tee $O/test.txt || exit 1
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 300 python -u tools/ab/w192_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.txt

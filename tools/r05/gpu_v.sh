#!/bin/bash
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_r256_gpu.py tests/test_gemm8p_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 600 python -u tools/ab/tile_graph_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/tile_graph_ab.txt
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 400 python -u tools/ab/kslope_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/kslope.txt

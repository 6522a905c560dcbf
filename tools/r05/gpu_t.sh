#!/bin/bash
# the 256-row 8-phase GEMM: path-equality tests, then the graph-replay A/B over the step's shapes
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8p_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so timeout -k 10 600 python -u tools/ab/tile_graph_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/tile_graph_ab.txt

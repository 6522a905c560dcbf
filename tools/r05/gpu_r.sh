#!/bin/bash
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "patch" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -u tools/ab/patch_bench.py 2>&1 | grep -v amdgpu.ids | tee $O/patch_bench.txt

#!/bin/bash
# r05 call F: the LN2 duplicate launch, row pattern and a quiet recomputation; patch embed / pack / CLIP tests
set -o pipefail
mkdir -p gpurun_out/r05f
env ICAP_SIDE_DW=1 PROBE_LN2_DUP=1 PROBE_CALLS=8 timeout -k 10 300 python -u tools/ab/det_probe5.py > gpurun_out/r05f/det_dup_rows.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05f/det_dup_rows.txt | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pack_gpu.py tests/test_kernels_gpu.py -k "pack or patch or im2col" > gpurun_out/r05f/tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r05f/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "clip or vit or dino" tests/test_bench_shape_gpu.py > gpurun_out/r05f/tests2.txt 2>&1
rc=$?
tail -5 gpurun_out/r05f/tests2.txt
exit $rc

#!/bin/bash
# r05 call E: LN2 inputs as read under the side-stream schedule; caption_pack multi-block kernel; fused patch embed
set -o pipefail
mkdir -p gpurun_out/r05e
env ICAP_SIDE_DW=1 PROBE_INPUT_CLONES=1 PROBE_LN2_DUP=1 timeout -k 10 300 python -u tools/ab/det_probe5.py > gpurun_out/r05e/det_clones.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05e/det_clones.txt | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pack_gpu.py tests/test_kernels_gpu.py -k "pack or patch or im2col" > gpurun_out/r05e/tests.txt 2>&1
rc=$?
tail -15 gpurun_out/r05e/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "clip or vit or dino" tests/test_bench_shape_gpu.py > gpurun_out/r05e/tests2.txt 2>&1
rc=$?
tail -15 gpurun_out/r05e/tests2.txt
exit $rc

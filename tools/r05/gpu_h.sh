#!/bin/bash
# r05 call H: LayerNorm-backward victim beside readers of its inputs; LN tests after the branch-free loads
set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 300 python -u tools/ab/ln_race_probe.py > gpurun_out/r05h/ln_race.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05h/ln_race.txt
[ $rc -eq 0 ] || exit $rc
PROBE_M=3200 timeout -k 10 300 python -u tools/ab/ln_race_probe.py > gpurun_out/r05h/ln_race_3200.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05h/ln_race_3200.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" tests/test_pack_gpu.py tests/test_grad_overwrite_gpu.py > gpurun_out/r05h/tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r05h/tests.txt
exit $rc

#!/bin/bash
# r05 call D: ds_bpermute victim beside each aggressor; GPU tests touched by the env-switch cleanup
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/ab/bperm_probe.py > gpurun_out/r05d/bperm.txt 2>&1; rc=$?
cat gpurun_out/r05d/bperm.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_lnfold_gpu.py tests/test_dp_nccl_gpu.py tests/test_determinism_gpu.py tests/test_grad_overwrite_gpu.py tests/test_pack_gpu.py > gpurun_out/r05d/tests.txt 2>&1
rc=$?
tail -15 gpurun_out/r05d/tests.txt
exit $rc

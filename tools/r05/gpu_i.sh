#!/bin/bash
# r05 call I: victim x aggressor matrix (which co-scheduled kernels corrupt which victims)
set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 600 python -u tools/ab/ln_race_probe.py > gpurun_out/r05i/matrix.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05i/matrix.txt
exit $rc

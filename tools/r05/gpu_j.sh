#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "attn or attention" > gpurun_out/r05j/attn_tests.txt 2>&1 || { tail -30 gpurun_out/r05j/attn_tests.txt; exit 1; }
tail -3 gpurun_out/r05j/attn_tests.txt
PROBE_VICTIMS=ln_bwd,ln_bwd_noparams,ln_bwd_nores,ln_bwd_bare PROBE_AGGRESSORS=none,tile,kout timeout -k 10 600 python -u tools/ab/ln_race_probe.py > gpurun_out/r05j/matrix.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05j/matrix.txt
exit $rc

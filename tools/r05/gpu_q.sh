#!/bin/bash
# the library without packed-FP32 instructions: the race tests, the model-level side-stream probe, LN race matrix
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_determinism_gpu.py tests/test_group_dw_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
PROBE_VICTIMS=ln_bwd,ln_bwd_bare,ln_fwd PROBE_AGGRESSORS=none,tile,kout,tile_nosplit PROBE_REPS=8 timeout -k 10 300 python -u tools/ab/ln_race_probe.py 2>&1 | grep -v amdgpu.ids > $O/ln_race.txt || { cat $O/ln_race.txt; exit 1; }
cat $O/ln_race.txt
ICAP_SIDE_DW=1 PROBE_CALLS=8 timeout -k 10 300 python -u tools/ab/det_probe5.py > $O/det_side.txt 2>&1 || { tail -20 $O/det_side.txt; exit 1; }
grep -E "RESULT|variant|differ|identical" $O/det_side.txt | head -20

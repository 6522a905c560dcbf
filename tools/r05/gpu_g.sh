#!/bin/bash
# r05 call G: side-stream determinism with the LayerNorm half-wave sums on DPP / permlane (no ds_bpermute)
set -o pipefail
mkdir -p gpurun_out/r05g
for v in "PROBE_LN2_DUP=1 PROBE_CALLS=8" "PROBE_CALLS=8" "PROBE_CALLS=6 ICAP_FUSED_SPLIT_K=0 ICAP_TRAIN_LN_FOLD=0"; do
  n=$(echo "$v" | tr '= ' '__')
  env ICAP_SIDE_DW=1 $v timeout -k 10 300 python -u tools/ab/det_probe5.py > gpurun_out/r05g/det_$n.txt 2>&1 || { echo "probe $n failed"; tail -20 gpurun_out/r05g/det_$n.txt; exit 1; }
  grep -E "RESULT|call|variant|layer" gpurun_out/r05g/det_$n.txt | head -30
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" tests/test_determinism_gpu.py tests/test_lnfold_gpu.py > gpurun_out/r05g/tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r05g/tests.txt
exit $rc

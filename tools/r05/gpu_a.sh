#!/bin/bash
# r05 call A: side-stream determinism localisation (4 variants) + configs[4] end-to-end test
set -o pipefail
mkdir -p gpurun_out/r05a
for v in "" "ICAP_FUSED_ACQUIRE=1" "ICAP_FUSED_SPLIT_K=0" "ICAP_SIDE_SERIAL=1"; do
  n=$(echo "${v:-base}" | tr '=' '_')
  env ICAP_SIDE_DW=1 $v timeout -k 10 240 python -u tools/ab/det_probe4.py > gpurun_out/r05a/det_$n.txt 2>&1 || { echo "probe $n failed rc=$?"; cat gpurun_out/r05a/det_$n.txt | tail -20; exit 1; }
  grep -E "RESULT|call|variant" gpurun_out/r05a/det_$n.txt
done
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_configs4_gpu.py > gpurun_out/r05a/configs4.txt 2>&1
rc=$?
tail -25 gpurun_out/r05a/configs4.txt
exit $rc

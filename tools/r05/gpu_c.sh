#!/bin/bash
# r05 call C: which part of the mapper LN2 backward varies under the side-stream schedule
set -o pipefail
mkdir -p gpurun_out/r05c
for v in "PROBE_LN2_DUP=1" "PROBE_LN_NOPARAMS=1" "PROBE_SYNC_LN2=1" "PROBE_B=128"; do
  n=$(echo "$v" | tr '= ' '__')
  env ICAP_SIDE_DW=1 $v timeout -k 10 240 python -u tools/ab/det_probe5.py > gpurun_out/r05c/det_$n.txt 2>&1 || { echo "probe $n failed rc=$?"; tail -20 gpurun_out/r05c/det_$n.txt; exit 1; }
  grep -E "RESULT|call|variant" gpurun_out/r05c/det_$n.txt
done

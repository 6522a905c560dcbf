#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/diag_pack.py > gpurun_out/diag1.log 2>&1; r1=$?
ICAP_FUSED_SPLIT_K=0 timeout -k 10 120 python3 -u tools/diag_pack.py > gpurun_out/diag0.log 2>&1
grep -v amdgpu gpurun_out/diag1.log gpurun_out/diag0.log

#!/bin/bash
# GEMM microbench under ICAP_GEMM_NARROW settings (128 x 64 tiles: 0 = off, 12 / 13 = forced) beside the default.
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-abn}; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/gemm_bench.py > $O/g_def.txt 2>&1 || exit 1
cols="<(grep -v amdgpu.ids $O/g_def.txt)"
for v in 0 12 13; do
  timeout -k 10 120 env ICAP_GEMM_NARROW=$v python -u tools/gemm_bench.py > $O/g_n$v.txt 2>&1 || { tail -5 $O/g_n$v.txt; exit 1; }
  cols="$cols <(grep -v amdgpu.ids $O/g_n$v.txt | awk '{print \$(NF-3), \$(NF-2)}')"
done
eval paste $cols | tee $O/gemm_narrow.txt

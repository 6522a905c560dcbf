#!/bin/bash
# GEMM microbench: default beside forced ICAP_GEMM_VARIANT values. usage: bash tools/ab_var.sh TAG v1 v2 ...
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-abv}; mkdir -p $O; shift
cd $R
timeout -k 10 120 python -u tools/gemm_bench.py > $O/g_def.txt 2>&1 || exit 1
cols="<(grep -v amdgpu.ids $O/g_def.txt)"
for v in "$@"; do
  timeout -k 10 120 env ICAP_GEMM_VARIANT=$v python -u tools/gemm_bench.py > $O/g_v$v.txt 2>&1 || { tail -5 $O/g_v$v.txt; exit 1; }
  cols="$cols <(grep -v amdgpu.ids $O/g_v$v.txt | awk '{print \$(NF-3), \$(NF-2)}')"
done
eval paste $cols | tee $O/gemm_var.txt

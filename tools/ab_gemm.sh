#!/bin/bash
# A/B of the GEMM microbench: the in-tree library vs another build (default: icap/libicap_hip_base.so),
# plus the in-tree library under each ICAP_GEMM_VARIANT given after the base path.
# usage: bash tools/ab_gemm.sh TAG [other.so [variant ...]]
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-ab}; mkdir -p $O
BASE=${2:-$R/gpt2-image-captioning_amd/icap/libicap_hip_base.so}
shift 2 2>/dev/null
cd $R
timeout -k 10 120 env ICAP_LIB=$BASE python -u tools/gemm_bench.py > $O/gemm_base.txt 2>&1 || { tail -5 $O/gemm_base.txt; exit 1; }
timeout -k 10 120 python -u tools/gemm_bench.py > $O/gemm_new.txt 2>&1 || { tail -5 $O/gemm_new.txt; exit 1; }
cols="<(grep -v amdgpu.ids $O/gemm_base.txt) <(grep -v amdgpu.ids $O/gemm_new.txt | awk '{print \$(NF-3), \$(NF-2), \$(NF-1), \$NF}')"
for v in "$@"; do
  timeout -k 10 120 env ICAP_GEMM_VARIANT=$v python -u tools/gemm_bench.py > $O/gemm_v$v.txt 2>&1 || { tail -5 $O/gemm_v$v.txt; exit 1; }
  cols="$cols <(grep -v amdgpu.ids $O/gemm_v$v.txt | awk '{print \$(NF-3), \$(NF-2)}')"
done
eval paste $cols | tee $O/gemm_ab.txt

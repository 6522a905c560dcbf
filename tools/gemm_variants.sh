#!/bin/bash
# GEMM variant sweep over the step's shapes (tools/gemm_bench.py), one process per variant.
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-gv}; mkdir -p $O
for v in ${VARIANTS:-default 0 4 5 9 1}; do
  if [ "$v" = default ]; then timeout -k 10 120 python $R/tools/gemm_bench.py > $O/v_$v.txt 2>&1 || exit 1
  else ICAP_GEMM_VARIANT=$v timeout -k 10 120 python $R/tools/gemm_bench.py > $O/v_$v.txt 2>&1 || exit 1; fi
done

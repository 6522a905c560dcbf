#!/bin/bash
# PMC pass (one counter set per run) of one GEMM shape per variant: bash tools/pmc_variants.sh TAG M N K "v1 v2 ..."
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$1; mkdir -p $O; M=$2; N=$3; K=$4
cd /tmp && export TMPDIR=/tmp
for v in $5; do
  ICAP_GEMM_VARIANT=$v timeout -k 10 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/a$v -o p -- python3 $R/tools/gemm_one.py $M $N $K 5 > $O/a$v.log 2>&1 || exit 1
  ICAP_GEMM_VARIANT=$v timeout -k 10 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $O/b$v -o p -- python3 $R/tools/gemm_one.py $M $N $K 5 > $O/b$v.log 2>&1 || exit 1
done
cd $R && for f in $(find $O -name '*.db'); do echo "== $f"; python tools/pmc_summary.py $f '%gemm%'; done > $O/summary.txt 2>&1

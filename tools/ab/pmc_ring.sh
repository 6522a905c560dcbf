#!/bin/bash
# counters of the N=768 long-K GEMM forms: the 4-stage ring (3584 rows, 168 tiles), the double-buffered tile kernel
# (8320 rows, 390 tiles) and the 256x256 8-phase kernel (8320 rows, 99 tiles)
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/pmc_ring; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
run() {  # tag M env pmc...
  local tag=$1 M=$2 envs=$3; shift 3
  env $envs timeout -s KILL 60 rocprofv3 --pmc "$@" -d $O/$tag -o p -- python3 $R/tools/gemm_one.py $M 768 3072 5 > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -3 $O/$tag.log; return 1; }
}
for form in "ring 3584 X=0" "nst2 8320 X=0" "g256 8320 GEMM_G256=1"; do
  set -- $form
  env $3 timeout -k 5 60 python3 $R/tools/gemm_one.py $2 768 3072 20 | tee $O/time_$1.txt || exit 1
  run ${1}_a $2 $3 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS || exit 1
  run ${1}_b $2 $3 TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  run ${1}_c $2 $3 TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || true
done
cd $R && for d in $O/*_[abc]; do f=$(ls $d/*.db 2>/dev/null | head -1); [ -n "$f" ] && { echo "== $(basename $d)"; python3 tools/pmc_summary.py $f "%gemm%"; }; done > $O/summary.txt 2>&1; cat $O/time_*.txt; cat $O/summary.txt | head -90

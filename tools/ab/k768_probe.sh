#!/bin/bash
# the plain 8320x2304x768 GEMM before (tools/ab_before: the build of 0c41ed9^, per-element
# activation switch) and after the epilogue change: event timing, then SQ instruction / wait counters per launch.
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/k768; mkdir -p $O; cd $R
for lib in current before; do
  if [ $lib == before ]; then export ICAP_LIB=$R/tools/ab_before/libicap_hip.so; else unset ICAP_LIB; fi
  timeout -k 10 60 python3 tools/gemm_one.py 8320 2304 768 50 | tee $O/time_$lib.txt || exit 1
  timeout -k 10 60 python3 tools/gemm_one.py 8320 2304 768 50 | tee -a $O/time_$lib.txt || exit 1
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a_$lib -o p -- python3 $R/tools/gemm_one.py 8320 2304 768 5 > $O/a_$lib.log 2>&1) || { tail -3 $O/a_$lib.log; exit 1; }
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $O/b_$lib -o p -- python3 $R/tools/gemm_one.py 8320 2304 768 5 > $O/b_$lib.log 2>&1) || { tail -3 $O/b_$lib.log; }
done
ls -R $O | head -30

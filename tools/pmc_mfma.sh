#!/bin/bash
# MFMA utilisation of the train step's kernels: one rocprofv3 PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
# GRBM_GUI_ACTIVE: 2 SQ + 1 GRBM slots) over a short graph-free bench run. usage: bash tools/pmc_mfma.sh TAG
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-pmc_mfma}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-graph --no-decode --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/m -o p -- python3 $B \
  > $O/m.log 2>&1 || { tail -5 $O/m.log; exit 1; }
cd $R && python tools/pmc_mfma.py $(find $O/m -name '*.db') > $O/pmc_mfma.txt && head -40 $O/pmc_mfma.txt

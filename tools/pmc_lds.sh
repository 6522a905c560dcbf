#!/bin/bash
# LDS bank conflicts of the train step's kernels: one rocprofv3 PMC pass (3 SQ slots) over a short graph-free bench
# run, then tools/pmc_mfma.sh's MFMA utilisation pass. usage: bash tools/pmc_lds.sh TAG
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-pmc_lds}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-graph --no-decode --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL -d $O/l -o p -- \
  python3 $B > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
cd $R && python tools/pmc_lds.py $(find $O/l -name '*.db') > $O/pmc_lds.txt && head -20 $O/pmc_lds.txt && rm -rf $O/l

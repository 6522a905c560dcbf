#!/bin/bash
# HBM traffic of the train step's kernels: separate FETCH_SIZE and WRITE_SIZE passes (TCC slots: 3 + 2) over a
# short graph-free bench run, plus a 1 GiB copy calibration. usage: bash tools/pmc_traffic.sh TAG
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/${1:-pmc_traffic}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-graph --no-decode --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/f -o p -- python3 $B > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/w -o p -- python3 $B > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/cf -o p -- python3 $R/tools/ab/copy_probe.py > $O/cf.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/cw -o p -- python3 $R/tools/ab/copy_probe.py > $O/cw.log 2>&1 || exit 1
cd $R && python tools/pmc_traffic.py $(find $O/f -name '*.db') $(find $O/w -name '*.db') $O/pmc_traffic.json \
  $(find $O/cf -name '*.db') $(find $O/cw -name '*.db')

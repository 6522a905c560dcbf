#!/bin/bash
# One GPU call: parity tests, bench (JSON line), rocprofv3 kernel stats of a short bench run.
# usage: bash tools/gpu_round.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
export TMPDIR=/tmp
echo "== pytest gpu" && timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1 ; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== bench" && ICAP_GEMM_DETAIL=$O/gemm_detail.txt timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kt -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R && python tools/kstats.py $(find $O/prof -name '*.db' | head -1) "bench.py --steps 5 --warmup 2 --no-decode (rocprofv3 kernel trace: 8 train steps = 1 eager warm-up + 5 timed graph replays + 1 graph warm-up... see bench.py; divide totals by 8)" > $O/kstats.txt 2>&1; head -40 $O/kstats.txt

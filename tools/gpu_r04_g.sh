#!/bin/bash
# round-4 pass G: every -m gpu test, the tile-kernel phase stamps (diagnostic library), the configs[3] bench line
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/${1:-r4g}; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/gemm_stamps.py > $O/stamps.txt 2>&1; rc=$?; cat $O/stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --config medium > $O/bench_medium.json 2> $O/bench_medium.err
rc=$?; tail -1 $O/bench_medium.json | cut -c1-600; [ $rc -eq 0 ] || { tail -5 $O/bench_medium.err; exit $rc; }

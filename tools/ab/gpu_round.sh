#!/bin/bash
# Full GPU pass (one gpurun call): every -m gpu test, then a default bench line. Stops at the first failing step.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/round; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|ERROR|bf16 |passed|failed" $O/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
tail -2 $O/bench.json; exit $rc

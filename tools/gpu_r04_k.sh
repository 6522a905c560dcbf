#!/bin/bash
# round-4 pass K: decode tests (ln_f folded into the LM head), the bench line, the NaN-aware side-stream probe, and
# a fresh PMC traffic summary of the train step's kernels
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/${1:-r4k}; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_lnfold_gpu.py tests/test_parity_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -1 $O/bench.json | cut -c1-300; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
ICAP_SIDE_DW=1 timeout -k 10 200 python -u tools/ab/det_probe2.py > $O/det2.txt 2>&1; rc=$?; grep "^call" $O/det2.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh $(basename $O)_pmc && head -c 1200 $R/gpurun_out/$(basename $O)_pmc/pmc_traffic.json

#!/bin/bash
# folded-LN decode GEMMs: kernel tests, decode tests, greedy A/B (ICAP_LN_FOLD=1 vs 0)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/lnfold; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_lnfold_gpu.py tests/test_parity_gpu.py -m gpu -x -v -k "fold or greedy or beam or topp" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|passed|failed" $O/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  ICAP_LN_FOLD=0 timeout -k 10 120 python -u tools/prof_decode.py 2>&1 | grep decode | sed 's/^/fused LN: /' || exit 1
  ICAP_LN_FOLD=1 timeout -k 10 120 python -u tools/prof_decode.py 2>&1 | grep decode | sed 's/^/folded LN: /' || exit 1
done

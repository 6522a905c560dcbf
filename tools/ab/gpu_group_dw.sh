#!/bin/bash
# grouped mapper dW (ICAP_GROUP_DW): its GPU tests, then the headline A/B against the serial split-K schedule
set -o pipefail
O=gpurun_out/gdw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_group_dw_gpu.py tests/test_grad_overwrite_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
bash tools/ab/train_ab.sh $O/ab base= group=ICAP_GROUP_DW=1 | tee $O/ab.txt

#!/bin/bash
# kernel + model GPU tests, then the step profile and bench line
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/quick; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
./tools/gpu_prof_step.sh

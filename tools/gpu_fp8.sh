#!/bin/bash
# MX fp8: the lane-map probe (host check runs on the CPU afterwards), then the fp8 kernel tests.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/fp8; mkdir -p $O; cd $R
timeout -k 10 60 ./tools/microbench/mx_probe $O/mx_probe.bin || exit $?
python tools/mx_probe_check.py $O/mx_probe.bin > $O/mx_probe_check.txt 2>&1; head -3 $O/mx_probe_check.txt
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|assert" $O/pytest.log | tail -12; exit $rc

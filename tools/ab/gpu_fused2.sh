#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_splitk_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/fused2.log 2>&1
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/fused2.log | head -40

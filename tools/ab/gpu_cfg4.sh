#!/bin/bash
# configs[4] pieces: DINOv3 / RoPE / GPT-2 large parity tests, then the configs[4] bench line and the headline line
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/cfg4; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v -k "dinov3 or rope or large" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large.json 2> $O/bench_large.err; rc=$?
tail -1 $O/bench_large.json; tail -3 $O/bench_large.err; exit $rc

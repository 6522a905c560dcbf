#!/bin/bash
# tower parity (CLIP / ViT-B/16 / DINOv3 pooled CLS vs HF) after the CLS-only last layer, then the configs[4] bench line
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/towers; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_model_gpu.py -m gpu -x -v -k "vit or dinov3 or clip" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config large --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_large.json 2> $O/bench_large.err; rc=$?
tail -1 $O/bench_large.json; tail -3 $O/bench_large.err; exit $rc

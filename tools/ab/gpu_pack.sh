#!/bin/bash
# packed token rows: the new kernels' GPU tests, the model/bench-shape parity tests, then a short bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_pack_gpu.py tests/test_model_gpu.py tests/test_bench_shape_gpu.py \
  -x -v --timeout 240 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep "" > gpurun_out/pack_bench.log 2>&1
rc=$?
tail -5 gpurun_out/pack_tests.log
tail -c 3000 gpurun_out/pack_bench.log
exit $rc

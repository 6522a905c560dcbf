#!/bin/bash
# batched transposes: kernel + model tests, then two bench lines
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/tbatch; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bench_shape_gpu.py tests/test_determinism_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|assert|passed|failed" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done

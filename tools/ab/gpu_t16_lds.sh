#!/bin/bash
# conflict-free read phase of the bf16 tile transpose: its tests, the LDS-conflict pass, the headline bench line
set -o pipefail
O=gpurun_out/t16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bench_shape_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_lds.sh t16/lds || exit 1
timeout -k 10 300 python -u bench.py --no-decode --no-cpu-baseline --sweep "" --no-unfrozen > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200

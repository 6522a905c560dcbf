#!/bin/bash
# K-outer transposed reads without bank conflicts: the K-outer / dW / trainer tests, the dW split sweep (compare
# profiles/r04_kout_split_sweep.txt), the LDS-conflict pass, the headline bench line
set -o pipefail
O=gpurun_out/klds; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_splitk_gpu.py tests/test_grad_overwrite_gpu.py tests/test_group_dw_gpu.py tests/test_bench_shape_gpu.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
SHAPES=none timeout -k 10 300 python -u tools/gemm_tiles_ab.py > $O/kout_sweep.txt 2>&1 || { tail -5 $O/kout_sweep.txt; exit 1; }
grep -v amdgpu.ids $O/kout_sweep.txt
bash tools/pmc_lds.sh klds/lds || exit 1
timeout -k 10 300 python -u bench.py --no-decode --no-cpu-baseline --sweep "" --no-unfrozen > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300

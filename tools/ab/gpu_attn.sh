#!/bin/bash
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/attn; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attention" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== new"; timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
echo "== old"; ICAP_LIB=$R/tools/ablib_att/libicap_old.so timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids

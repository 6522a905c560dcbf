#!/bin/bash
# specialised activation epilogues: the activated-product probe and the step with ICAP_SPEC_ACT = 1 / 0, then the
# GEMM / model GPU tests
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/specact; mkdir -p $O; cd $R
for v in 1 0; do
  ICAP_SPEC_ACT=$v timeout -k 10 200 python -u tools/act_cost_probe.py 2>&1 | grep -v amdgpu | sed "s/^/spec=$v /" || exit 1
done
for v in 1 0 1 0; do
  ICAP_SPEC_ACT=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('spec=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_ms_per_step'])"
done
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_parity_gpu.py tests/test_fused_splitk_gpu.py tests/test_pack_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAIL|Error|assert|passed|failed" $O/pytest.log | tail -12; exit $rc

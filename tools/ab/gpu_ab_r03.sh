#!/bin/bash
# A/B of the current build against tools/ab_cur (the previous build): attention and GEMM microbenchmarks, then the
# kernel / model GPU tests and the bench line.
R=$(cd "$(dirname "$0")/.." && pwd); O=$R/gpurun_out/ab; mkdir -p $O; cd $R
rm -f $O/*.txt
for i in 1 2; do
  ICAP_LIB=$R/tools/ab_cur/libicap_hip.so timeout -k 10 60 python3 tools/attn_bench.py 2>&1 | grep attn | sed 's/^/before /' | tee -a $O/attn.txt || exit 1
  timeout -k 10 60 python3 tools/attn_bench.py 2>&1 | grep attn | sed 's/^/after  /' | tee -a $O/attn.txt || exit 1
done
ICAP_LIB=$R/tools/ab_cur/libicap_hip.so timeout -k 10 200 python3 tools/gemm_bench.py > $O/gemm_before.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/gemm_bench.py > $O/gemm_after.txt 2>&1 || exit 1
paste -d'|' <(cut -c1-60 $O/gemm_before.txt) <(cut -c40-60 $O/gemm_after.txt) | head -30
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_gemm256_gpu.py tests/test_fp8_gpu.py tests/test_bench_shape_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --sweep "" > $O/bench.json 2> $O/bench.err; rc=$?; tail -1 $O/bench.json | cut -c1-250; exit $rc

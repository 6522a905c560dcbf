set -o pipefail
mkdir -p gpurun_out/ring1
timeout -k 10 300 python -u -m pytest tests/test_gemm_ring_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/ring1/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/ring1/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/ring1/gemm_bench.txt 2>&1; cat gpurun_out/ring1/gemm_bench.txt

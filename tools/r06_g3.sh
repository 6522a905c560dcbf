set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_roles_gpu.py tests/test_gemm_w192_gpu.py tests/test_gemm256_gpu.py tests/test_fused_splitk_gpu.py tests/test_lnfold_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.txt 2>&1 || { tail -30 $O/gemm_tests.txt; exit 1; }
tail -2 $O/gemm_tests.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/roles_ab.txt 2>&1; cut -c1-120 $O/roles_ab.txt

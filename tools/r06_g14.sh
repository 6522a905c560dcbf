# round 6: variant 32 (160 x 128 split-role tiles): roles parity tests, the GEMM tests the automatic plan touches, the A/B table
set -o pipefail
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_roles_gpu.py tests/test_gemm_w192_gpu.py tests/test_lnfold_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -3 $O/test.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-150 $O/ab.txt

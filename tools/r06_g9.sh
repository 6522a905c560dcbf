# round 6: the K-outer split-role GEMM (variant 31): parity tests, then the dW A/B
set -o pipefail
O=gpurun_out/r06g9; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gemm_roles_kout_gpu.py -x -v --timeout 60 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -3 $O/test.txt
timeout -k 10 200 python -u tools/ab/dw_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt

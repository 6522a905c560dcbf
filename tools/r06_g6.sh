# round 6: the two-per-CU split-role kernel (variant 29): its parity tests, then the A/B table
set -o pipefail
O=gpurun_out/r06g6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_roles_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-140 $O/ab.txt

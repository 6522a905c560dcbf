# round 6: the persistent split-role GEMM with the overlapped epilogue (variant 30): parity tests, then the A/B table
set -o pipefail
O=gpurun_out/r06g7; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gemm_pers_gpu.py -x -v --timeout 60 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -3 $O/test.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-150 $O/ab.txt
timeout -k 10 120 python -u tools/ab/pers_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt

# round 6: variant 28 on 32-deep stages (5-stage ring): roles parity tests, the A/B table and the stamps
set -o pipefail
O=gpurun_out/r06g11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_roles_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-140 $O/ab.txt
timeout -k 10 120 python -u tools/ab/roles_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt

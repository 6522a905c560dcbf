# round 6: caller split-K on the split-role rings: parity test, then the LM head dX A/B
set -o pipefail
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_roles_gpu.py -x -q -k "split_k" --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/lmhead_dx_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt

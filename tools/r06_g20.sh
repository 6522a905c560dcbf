# round 6: LN parameter reduce with its row loads in flight together; decode LM head back on the tile loop: the
# kernels / determinism / group-dW / decode tests, the LM head probe and the greedy rate
set -o pipefail
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_group_dw_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/lmhead_dx_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -7 $O/ab.txt
timeout -k 10 300 python -u tools/prof_decode.py > $O/greedy.txt 2>&1 || { tail -20 $O/greedy.txt; exit 1; }
tail -1 $O/greedy.txt

# round 6: folded-LN decode GEMMs with the W row sums prefetched: decode parity tests, decode microbench, greedy rate
set -o pipefail
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lnfold_gpu.py tests/test_parity_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/decode_bench.py > $O/dec.txt 2>&1 || { tail -20 $O/dec.txt; exit 1; }
cat $O/dec.txt
timeout -k 10 300 python -u tools/prof_decode.py > $O/greedy.txt 2>&1 || { tail -20 $O/greedy.txt; exit 1; }
tail -3 $O/greedy.txt

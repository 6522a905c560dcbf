# round 6: decode weight prefetch: decode parity tests, then the A/B in one process
set -o pipefail
O=gpurun_out/g18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lnfold_gpu.py tests/test_parity_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/decode_prefetch_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt

# round 6: batched LN parameter reduces of the mapper backward: bitwise test, mapper / trainer tests, step A/B vs the tree
set -o pipefail
O=gpurun_out/g24; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_group_dw_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 400 python -u tools/ab/ln_param_batch_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt

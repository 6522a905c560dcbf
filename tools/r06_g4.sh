set -o pipefail
O=gpurun_out/${1:-r06d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_roles_gpu.py -x -q --timeout 120 --timeout-method thread > $O/roles_tests.txt 2>&1 || { tail -30 $O/roles_tests.txt; exit 1; }
tail -2 $O/roles_tests.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/roles_ab.txt 2>&1; cut -c1-150 $O/roles_ab.txt

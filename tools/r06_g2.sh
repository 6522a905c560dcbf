set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
cd tools/microbench && timeout -k 10 100 ./gemm_lab 9 > ../../$O/lab9.txt 2>&1 && timeout -k 10 120 ./gemm_lab > ../../$O/lab_all.txt 2>&1; cd ../..
timeout -k 10 300 python -u -m pytest tests/test_gemm_roles_gpu.py -x -v --timeout 120 --timeout-method thread > $O/roles_tests.txt 2>&1 || { tail -30 $O/roles_tests.txt; exit 1; }
tail -3 $O/roles_tests.txt
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/roles_ab.txt 2>&1; cat $O/roles_ab.txt | cut -c1-140

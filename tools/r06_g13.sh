# round 6: the grouped K-outer launch (icap_gemm_group) and the fused mapper schedule: parity tests, then the step A/B
set -o pipefail
O=gpurun_out/r06g13; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_roles_kout_gpu.py tests/test_group_dw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/mapper_dw_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt

set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/gv2; mkdir -p $O; cd $R
for v in 10 11; do ICAP_GEMM_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 60 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -30 $O/test_$v.log; exit 1; }; tail -1 $O/test_$v.log; done
VARIANTS="default 10 11" bash tools/gemm_variants.sh gv2

# round 6: variant 30 stamps with and without the epilogue waves' stores (timing diagnostic build)
set -o pipefail
O=gpurun_out/r06g8; mkdir -p $O
timeout -k 10 120 python -u tools/ab/pers_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_diag.so timeout -k 10 120 python -u tools/ab/pers_stamps.py > $O/stamps_noepi.txt 2>&1 || { tail -20 $O/stamps_noepi.txt; exit 1; }
cat $O/stamps_noepi.txt

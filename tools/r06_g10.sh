# round 6: attention forward with batched K/V staging and the key mask in LDS — parity tests, then old vs new timing
set -o pipefail
O=gpurun_out/r06g10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_pack_gpu.py -x -q -k "attn or attention or pack" --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
ICAP_LIB=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_old.so timeout -k 10 120 python -u tools/ab/attn_step_probe.py > $O/old.txt 2>&1 || { tail -20 $O/old.txt; exit 1; }
timeout -k 10 120 python -u tools/ab/attn_step_probe.py > $O/new.txt 2>&1 || { tail -20 $O/new.txt; exit 1; }
echo old; cat $O/old.txt; echo new; cat $O/new.txt

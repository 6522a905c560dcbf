# round 6: attention forward v2 with all its loads in one round trip (branch-free Q / K / V / key-mask loads, key mask
# in LDS): attention parity tests, then the step-shape attention probe
set -o pipefail
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pack_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 300 python -u tools/ab/attn_step_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt

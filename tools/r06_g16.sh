# round 6: LM head dX / decode LM head forms; decode per-kernel microbench
set -o pipefail
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 300 python -u tools/ab/lmhead_dx_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 python -u tools/decode_bench.py > $O/dec.txt 2>&1 || { tail -20 $O/dec.txt; exit 1; }
cat $O/dec.txt

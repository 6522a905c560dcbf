#!/bin/bash
# L2 channel-stride probe: the step's GEMM shapes with A/B rows padded by PAD elements (row stride no longer a
# multiple of the power-of-two channel interleave)
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/gpurun_out/pad
for pad in 0 64 8 128; do
  PAD=$pad REPS=10 timeout -k 10 300 python -u $R/tools/gemm_bench.py > $R/gpurun_out/pad/pad$pad.txt 2>&1 || exit 1
  echo "== pad $pad"; grep -E "x  3072 |x  2304 |x   768 plain|sum" $R/gpurun_out/pad/pad$pad.txt | head -14
done

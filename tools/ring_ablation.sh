#!/bin/bash
# Diagnostic: build the library with the ring kernel's MFMAs / LDS-DMA / fragment reads removed (ICAP_RING_ABL)
# and time the GEMM shapes with each (tools/gemm_bench.py via ICAP_LIB). Build here (CPU), run on the GPU box.
#   build:  bash tools/ring_ablation.sh build      run:  bash tools/ring_ablation.sh run
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/gpt2-image-captioning_amd/csrc
if [ "$1" = build ]; then
  for a in 1 2 3; do
    mkdir -p /tmp/abl$a
    for f in runtime gemm layernorm attention attention_mfma elementwise preprocess; do
      extra=""; [ $f = gemm ] && extra="-DICAP_RING_ABL=$a"
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include -munsafe-fp-atomics $extra -c $CS/$f.hip -o /tmp/abl$a/$f.o &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/ablibs/libicap_abl$a.so /tmp/abl$a/*.o
  done
else
  mkdir -p $R/gpurun_out/abl
  for a in 0 1 2 3; do
    lib=""; [ $a != 0 ] && lib=$R/tools/ablibs/libicap_abl$a.so
    ICAP_LIB=$lib REPS=10 timeout -k 10 300 python -u $R/tools/gemm_bench.py > $R/gpurun_out/abl/abl$a.txt 2>&1
    echo "== ablation $a"; grep -E "8320x   768x  3072 plain|8320x  3072x   768 gelu|3200x   768x  3072 plain|sum" $R/gpurun_out/abl/abl$a.txt
  done
fi

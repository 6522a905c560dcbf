#!/bin/bash
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
PROBE_VICTIMS=ln_bwd_bare PROBE_AGGRESSORS=tile,tile_nosplit,kout,kout_nosplit,g256,skinny PROBE_REPS=8 timeout -k 10 300 python -u tools/ab/ln_race_probe.py 2>&1 | grep -v amdgpu.ids | grep -v "fit:\|first wrong" > $O/aggr.txt || { cat $O/aggr.txt; exit 1; }
cat $O/aggr.txt
for L in product nopk_all; do
  lib=""; [ $L = nopk_all ] && lib=tools/ab/_libs/libicap_nopk_all.so
  ICAP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$L.json 2> $O/bench_$L.err || { tail -20 $O/bench_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$L.json')); r=d['roofline']; print('$L', d['value'], d['ms_per_step'], r['frac'], r['gpt2_block']['ms'], d['greedy_captions_per_s'], d['train_unfrozen']['images_per_s'])"
done

#!/bin/bash
# LN backward side-stream victim: half-wave reduction variants (ICAP_LIB = diagnostic builds, -DICAP_LN_HSUM_DIAG=n)
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
export PROBE_VICTIMS=ln_bwd_bare PROBE_AGGRESSORS=none,tile,kout PROBE_REPS=8
for v in product hs1 hs2 hs3 hs4; do
  case $v in
    product) L=""; d="product: DPP + permlane16_swap";;
    hs1) L=tools/ab/_libs/libicap_hs1.so; d="s_nop 7 between permlane16_swap and its add";;
    hs2) L=tools/ab/_libs/libicap_hs2.so; d="__shfl_xor butterfly (ds_bpermute, round 4)";;
    hs3) L=tools/ab/_libs/libicap_hs3.so; d="64 v_readlane, no cross-lane VALU/LDS op";;
    hs4) L=tools/ab/_libs/libicap_hs4.so; d="s_nop 7 around every DPP step and the swap";;
  esac
  echo "== $v: $d" >> $O/matrix.txt
  ICAP_LIB=$L timeout -k 10 300 python -u tools/ab/ln_race_probe.py 2>&1 | grep -v amdgpu.ids | grep -v "fit:" >> $O/matrix.txt || { cat $O/matrix.txt; exit 1; }
done
cat $O/matrix.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], r['frac'], r['gpt2_block'], r['replay_roofline'], r['eager_roofline'])"

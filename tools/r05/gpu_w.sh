#!/bin/bash
# unsplit 192 x 64 ring for the short fused launches: the whole GPU suite, then the step with / without that rule
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
S=$PWD/gpt2-image-captioning_amd/icap/libicap_hip_stamps.so
for r in 1 2; do
  for m in 0 3; do
    ICAP_W192=$m ICAP_LIB=$S timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --sweep "" > $O/bench_w$m.$r.json 2> $O/bench_w$m.$r.err || { tail -20 $O/bench_w$m.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench_w$m.$r.json')); print('W192=$m', d['value'], d['ms_per_step'], d.get('ms_per_step_median'))"
  done
done

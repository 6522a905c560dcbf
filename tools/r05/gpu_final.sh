#!/bin/bash
# final tree: the whole GPU suite, smoke(), and the default bench line
set -o pipefail
O=gpurun_out/r05final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -3
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['gpt2_block']['frac'], d['greedy_captions_per_s'], r['traffic'], r['traffic_source'])"

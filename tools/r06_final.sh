# round 6 closing run: full GPU suite, smoke(), the default bench line, then the greedy-decode kernel table
set -o pipefail
O=gpurun_out/${1:-r06final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -40 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['gpt2_block']['frac'], d['greedy_captions_per_s'], r['kernel'])"
R=$PWD; cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dp -o run -- python3 -u tools/prof_decode.py > $O/dec.log 2>&1 || { tail -20 $O/dec.log; exit 1; }
tail -1 $O/dec.log
db=$(find $O/dp -name "run_results.db" | head -1)
python tools/kstats.py $db "greedy decode (tools/prof_decode.py: B = 128, 50 tokens, bf16, graph replay; 2 warm-up + 5 timed generate calls) under rocprofv3 --kernel-trace" > $O/dec_kstats.txt && head -20 $O/dec_kstats.txt | cut -c1-160
rm -rf $O/dp

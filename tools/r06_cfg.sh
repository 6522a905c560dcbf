# round 6: configs[3] (medium) and configs[4] (large, fp8 MX) bench lines on the closing tree
set -o pipefail
O=gpurun_out/r06cfg; mkdir -p $O
timeout -k 10 500 python -u bench.py --config medium --no-cpu-baseline > $O/medium.json 2> $O/medium.err || { tail -20 $O/medium.err; exit 1; }
python -c "import json; d=json.load(open('$O/medium.json')); print('medium', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('greedy_captions_per_s'))"
timeout -k 10 500 python -u bench.py --config large --fp8 --no-cpu-baseline > $O/large.json 2> $O/large.err || { tail -20 $O/large.err; exit 1; }
python -c "import json; d=json.load(open('$O/large.json')); print('large fp8', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('greedy_captions_per_s'))"

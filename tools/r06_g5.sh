set -o pipefail
O=gpurun_out/${1:-r06f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bf16w_gpu.py "tests/test_parity_gpu.py::test_vit_extract_directory_end_to_end" -v -s --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|bf16|bench128|greedy|Error|assert" $O/tests.txt | head -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/ab/patch_bench.py > $O/patch.txt 2>&1 && cat $O/patch.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['gpt2_block']['frac'], d['greedy_captions_per_s'], d['clip_extraction'])"

set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/medium1; mkdir -p $O; cd $R; export TMPDIR=/tmp
ICAP_GEMM_DETAIL=$O/gemm_detail.txt timeout -k 10 400 python -u bench.py --config medium > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt -- python3 $R/bench.py --config medium --steps 5 --warmup 2 --no-cpu-baseline --no-decode > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R && python tools/kstats.py $(find $O/prof -name '*.db' | head -1) "bench.py --config medium --steps 5 --warmup 2 --no-decode (rocprofv3 kernel trace; 8 train steps incl. warm-ups, divide by 8)" > $O/kstats.txt 2>&1; head -25 $O/kstats.txt

# kernel table of the timed train steps (rocprofv3 kernel trace, window between optimizer launches)
set -o pipefail
O=gpurun_out/${1:-r06prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
db=$(find $O/p -name "run_results.db" | head -1)
python tools/kstats.py $db "the 10 timed train steps of 'bench.py --steps 10 --warmup 3 --no-decode --no-cpu-baseline --sweep \"\"' (packed B = 128, graph replay): kernels between the end of the 3rd and the 13th optimizer launch" --window adam_update_kernel 3 10 > $O/kstats.txt && head -45 $O/kstats.txt | cut -c1-170
rm -rf $O/p

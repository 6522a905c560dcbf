# round 6: fresh kernel window of the current tree, then the N = 2 data-parallel rehearsal (both ranks on cuda:0 over gloo)
set -o pipefail
bash tools/r06_prof.sh r06prof3 || exit 1
O=gpurun_out/r06dp; mkdir -p $O
ICAP_BENCH_DP_REHEARSAL=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --no-decode --no-cpu-baseline --sweep "" > $O/dp.json 2> $O/dp.err || { tail -30 $O/dp.err; exit 1; }
tail -c 600 $O/dp.json

#!/bin/bash
# round-4 GPU pass: every -m gpu test, the default bench line (with the per-shape GEMM / attention table of its
# eager roofline pass), and a rocprofv3 kernel-time table of the packed train step. Stops at the first failing step.
# usage: tools/gpu_r04.sh TAG [quick|skip-tests|full] [bench-only]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); T=${1:-r4}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export PYTHONUNBUFFERED=1
if [ "$2" = "quick" ]; then  # the tests of this round's changes only
  timeout -k 10 600 python -u -m pytest tests/test_lnfold_gpu.py tests/test_fused_splitk_gpu.py tests/test_configs3_gpu.py tests/test_pack_gpu.py tests/test_determinism_gpu.py tests/test_bench_shape_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
elif [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
fi
ICAP_GEMM_DETAIL=$O/gemm_detail.txt timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -1 $O/bench.json | cut -c1-400; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
[ "$3" = "bench-only" ] && exit 0
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 8 --warmup 3 --no-decode --no-cpu-baseline --sweep "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cd $R && python tools/kstats.py $O/p/run_results.db "the 8 timed train steps of 'bench.py --steps 8 --warmup 3 --no-decode --sweep \"\"' (packed B = 128, graph replay): kernels between the end of the 3rd and the 11th optimizer launch" --window adam_update_kernel 3 8 > $O/kstats.txt && head -16 $O/kstats.txt | cut -c1-150
python tools/kstats.py $O/p/run_results.db "whole 'bench.py --steps 8 --warmup 3 --no-decode --sweep \"\"' run: model build (one-time: the fp32 GEMMs are the LayerNorm folds of the frozen weights), then the packed train step x 12 (3 warm-up + 8 timed + 1 eager roofline pass)" > $O/kstats_run.txt
rm -rf $O/p
if [ -z "$SKIP_DIAG" ]; then
  timeout -k 10 300 python -u tools/gemm_diag.py > $O/gemm_diag.txt 2>&1 || { tail -5 $O/gemm_diag.txt; exit 1; }
  cat $O/gemm_diag.txt
  timeout -k 10 300 python -u tools/gemm_tiles_ab.py > $O/gemm_tiles_ab.txt 2>&1 || { tail -5 $O/gemm_tiles_ab.txt; exit 1; }
  cat $O/gemm_tiles_ab.txt
fi
if [ -n "$TRAIN_AB" ]; then  # e.g. TRAIN_AB='base= fold0=ICAP_TRAIN_LN_FOLD=0'
  bash tools/ab/train_ab.sh $O/train_ab $TRAIN_AB | tee $O/train_ab.txt || exit 1
fi
# side-stream determinism probes (diagnostic; failures here do not stop the pass)
for d in ${DET_DIAGS:-none scratch no_dw no_db}; do
  ICAP_SIDE_DW=1 ICAP_SIDE_DIAG=${d%%+*} PROBE_DW_SPLIT=$([ "${d#*+}" = "split1" ] && echo 1) timeout -k 10 200 python -u tools/ab/det_probe2.py > $O/det_$d.txt 2>&1
  rc=$?; echo "== side diag $d (rc $rc)"; grep "^call" $O/det_$d.txt | cut -c1-200
  [ $rc -eq 0 ] || exit $rc  # a probe that crashed or timed out ends the pass
done

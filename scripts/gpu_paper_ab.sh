#!/bin/bash
# GogoroPaper iteration: the paper (and physics) GPU tests, then an A/B of the
# step with the per-link force reduction inside the post launch (default) and
# as its own launch (TG_PAPER_RB_LAUNCH=1), twice each, and a rocprofv3 summary.
# Every GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/paper_ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_paper.py tests/test_gpu_physics.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do  # f=1: the rigid-body force reduction as its own launch
    TG_PAPER_RB_LAUNCH=$f timeout -k 10 200 python bench.py --task GogoroPaper --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/bench_f${f}_$r.log 2>&1 || exit $?
    echo "rb_launch=$f run $r: $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*' $OUT/bench_f${f}_$r.log | tr '\n' ' ')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --task GogoroPaper --steps 300 --warmup 50 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
cut -d, -f1-4 $OUT/trace/run_kernel_stats.csv | head -8
exit 0

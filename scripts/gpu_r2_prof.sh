#!/bin/bash
# Round-2 evidence session: Gogoro bench line, rocprofv3 kernel statistics and
# FETCH/WRITE PMC passes of the two headline workloads, SQ counter passes of
# the ThormangWalk step kernel.  Every GPU step has its own time limit; a
# failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/r2prof}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --task Gogoro > $OUT/bench_gogoro4096.log 2>&1 || exit $?
tail -c 400 $OUT/bench_gogoro4096.log
PROF_DIR=$OUT/prof_thormangwalk4096 BENCH_ARGS="--task ThormangWalk --steps 200 --warmup 30" bash scripts/gpu_profile.sh > $OUT/prof_t.log 2>&1 || exit $?
PROF_DIR=$OUT/prof_gogoro4096 BENCH_ARGS="--task Gogoro --steps 200 --warmup 30" bash scripts/gpu_profile.sh > $OUT/prof_g.log 2>&1 || exit $?
echo profiles ok
PROF_DIR=$OUT/sq_thormangwalk4096 BENCH_ARGS="--task ThormangWalk --steps 100 --warmup 20" bash scripts/gpu_pmc_sq.sh > $OUT/sq_t.log 2>&1 || exit $?
PROF_DIR=$OUT/sq_gogoro4096 BENCH_ARGS="--task Gogoro --steps 100 --warmup 20" bash scripts/gpu_pmc_sq.sh > $OUT/sq_g.log 2>&1 || exit $?
echo sq ok
exit 0

#!/bin/bash
# Round-end evidence on one GPU box: the bench line of every workload in
# DESIGN.md §5, rocprofv3 kernel statistics + FETCH/WRITE PMC passes of the two
# headline workloads, and the step kernel's section profile.  Every GPU step
# has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/refresh}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$n.log 2>&1
  local rc=$?; echo "bench $n rc=$rc $(tail -c 300 $OUT/bench_$n.log | grep -o '"value": [0-9.e+]*' | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
run thormangwalk4096 --task ThormangWalk
run thormangwalkdr4096 --task ThormangWalkDR --no-cpu-baseline
run thormangwalk8192 --task ThormangWalk --num-envs 8192 --no-cpu-baseline
run thormangwalk16384 --task ThormangWalk --num-envs 16384 --no-cpu-baseline
run thormangwalkdr16384 --task ThormangWalkDR --num-envs 16384 --no-cpu-baseline
run gogoro4096 --task Gogoro
run gogoro4096_terrain --task Gogoro --terrain
run gogoropaper2048 --task GogoroPaper --num-envs 2048 --no-cpu-baseline
run gogoropaper4096 --task GogoroPaper --no-cpu-baseline
PROF_DIR=$OUT/prof_thormangwalk4096 BENCH_ARGS="--task ThormangWalk --steps 200 --warmup 30" bash scripts/gpu_profile.sh > $OUT/prof_t.log 2>&1 || exit $?
PROF_DIR=$OUT/prof_gogoro4096 BENCH_ARGS="--task Gogoro --steps 200 --warmup 30" bash scripts/gpu_profile.sh > $OUT/prof_g.log 2>&1 || exit $?
echo profiles ok
PROF_DIR=$OUT/sq_thormangwalk4096 BENCH_ARGS="--task ThormangWalk --steps 100 --warmup 20" bash scripts/gpu_pmc_sq.sh > $OUT/sq_t.log 2>&1 || exit $?
PROF_DIR=$OUT/sq_gogoro4096 BENCH_ARGS="--task Gogoro --steps 100 --warmup 20" bash scripts/gpu_pmc_sq.sh > $OUT/sq_g.log 2>&1 || exit $?
echo sq ok
if [ -f thormang_isaacgym_amd/libtgsim_prof.so ]; then
  for t in ThormangWalk Gogoro; do
    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_prof.so timeout -k 10 120 python scripts/section_prof.py $t > $OUT/section_$t.txt 2>&1 || exit $?
  done
  echo sections ok
fi
exit 0

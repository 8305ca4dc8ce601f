# shared-cache A/B + HBM traffic of the current build (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3j; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_physics.py tests/test_gpu_edge.py -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
for t in ThormangWalk ThormangWalkDR; do
  timeout -k 10 300 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_$t.log 2>&1 || exit $?
  TG_NO_SHARED_CACHE=1 timeout -k 10 300 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_own.log 2>&1 || exit $?
  echo "$t shared $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_$t.log) own $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_own.log)"
done
PROF_DIR=$OUT/prof_walk BENCH_ARGS="--task ThormangWalk --steps 200 --warmup 30" timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/prof_walk.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $OUT/prof_walk > $OUT/pmc_walk.json
TG_NO_SHARED_CACHE=1 PROF_DIR=$OUT/prof_walk_own BENCH_ARGS="--task ThormangWalk --steps 200 --warmup 30" timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/prof_walk_own.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $OUT/prof_walk_own > $OUT/pmc_walk_own.json
grep -h '"hbm_bytes_per_dispatch"' $OUT/pmc_walk.json $OUT/pmc_walk_own.json

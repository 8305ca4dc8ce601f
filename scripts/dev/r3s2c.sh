# developer A/B session: the named test files on the current library, then each library in LIBS over TASKS (two reps)
set -u
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/ab}; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for task in ${TASKS:-ThormangWalk Gogoro}; do
    for lib in ${LIBS:-libtgsim.so libtgsim_base.so}; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $task --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/ab_${task}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $task $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/ab_${task}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

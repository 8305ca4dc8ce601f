# developer session: the GPU suite after the TGS / rounding-control changes, then A/B against the pre-TGS library
set -u
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/s5}; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" $OUT/tests.log | tail -15; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for task in ThormangWalk Gogoro; do
    for lib in libtgsim.so libtgsim_pgs.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $task --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/ab_${task}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $task $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/ab_${task}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

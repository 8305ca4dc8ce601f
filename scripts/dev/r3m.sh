# segments (pass 1a + pass 3) correctness + A/B; store/read split of a schedule step (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3m; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for t in ThormangWalk Gogoro; do
    for lib in libtgsim_seg0.so libtgsim_seg1.so libtgsim_seg4.so libtgsim_seg5.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $t $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_${lib}_$rep.log)"
    done
  done
  for lib in libtgsim_dk1.so libtgsim_dk2.so libtgsim_dk3.so libtgsim_dk4.so; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task ThormangWalk --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${lib}_$rep.log 2>&1 || exit $?
    echo "$rep $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${lib}_$rep.log)"
  done
done

# 2b-segment JIT mismatch bisect; NoPost compiled path vs the oracle; section profiles seg vs not; velocity-iteration cost
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3o; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in libtgsim_seg2.so libtgsim_seg2nm.so; do
  TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_physics.py -m gpu -q --timeout 200 --timeout-method thread -k "runtime_specialisation" > $OUT/jit_$lib.log 2>&1
  rc=$?; echo "$lib jit rc=$rc $(grep -o "AssertionError: .*" $OUT/jit_$lib.log | head -1)"; [ $rc -le 1 ] || exit $rc
done
TG_WALK_UNFUSED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity_long.py -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/walk_unfused.log 2>&1
rc=$?; echo "walk unfused rc=$rc"; grep -E "FAILED|passed|failed" $OUT/walk_unfused.log | tail -5; [ $rc -le 1 ] || exit $rc
for t in ThormangWalk Gogoro; do
  for lib in libtgsim_prof0.so libtgsim_prof.so; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python scripts/section_prof.py $t > $OUT/section_${t}_$lib.txt 2>&1 || exit $?
  done
  paste $OUT/section_${t}_libtgsim_prof0.so.txt $OUT/section_${t}_libtgsim_prof.so.txt | grep -v Warn | grep "%" | head -20
done
for t in ThormangWalk Gogoro; do
  timeout -k 10 300 python scripts/dev/viters_cost.py $t > $OUT/viters_$t.txt 2>&1 || exit $?
  tail -3 $OUT/viters_$t.txt
done

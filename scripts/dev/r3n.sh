# segment passes: JIT-vs-compiled bisect, then the full GPU suite on the all-segment build (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3n; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in libtgsim_seg0.so libtgsim_seg1.so libtgsim_seg4.so libtgsim_seg2.so libtgsim_seg8.so libtgsim.so; do
  TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_physics.py -m gpu -q --timeout 200 --timeout-method thread -k "runtime_specialisation" > $OUT/jit_$lib.log 2>&1
  rc=$?; echo "$lib jit rc=$rc $(grep -o "AssertionError: .*" $OUT/jit_$lib.log | head -1)"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=8 -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -12; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for t in ThormangWalk Gogoro; do
    for lib in libtgsim_seg0.so libtgsim_seg2.so libtgsim_seg8.so libtgsim.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $t $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_${lib}_$rep.log)"
    done
  done
done
for n in 1024 4096; do
  for lib in libtgsim.so libtgsim_epb4.so libtgsim_epb8.so; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task ThormangWalk --num-envs $n --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_n${n}_${lib}.log 2>&1 || exit $?
    echo "N=$n $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_n${n}_${lib}.log)"
  done
done

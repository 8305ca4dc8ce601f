# full GPU suite on the lane-pair scooters, then env-stride pad A/B for them (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3x; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
  for task in Gogoro GogoroPaper; do
    for lib in libtgsim.so libtgsim_pad0.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $task --num-envs 4096 --steps 500 --warmup 50 --no-cpu-baseline > $OUT/bench_${task}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $task $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_${task}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

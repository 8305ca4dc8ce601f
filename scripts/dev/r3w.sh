# Gogoro with lane-pair (16 lanes per env) scheduling: parity + A/B (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3w; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_pair4.so timeout -k 10 300 python -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gogoro.py tests/test_gpu_paper.py > $OUT/tests_pair4.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests_pair4.log; exit 1; }
tail -2 $OUT/tests_pair4.log
for rep in 1 2; do
  for task in Gogoro GogoroPaper; do
    for lib in libtgsim.so libtgsim_pair4.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $task --num-envs 4096 --steps 500 --warmup 50 --no-cpu-baseline > $OUT/bench_${task}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $task $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_${task}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

# kernel start: table loads in one round trip, walk pre-physics outputs stored by the epilogue, state loads batched (A/B + tests)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3u; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_physics.py tests/test_gpu_edge.py tests/test_gpu_parity_long.py -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -8; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for t in ThormangWalk ThormangWalkDR Gogoro; do
    for lib in libtgsim_prevk.so libtgsim.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $t $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

# ES pad-2 (Thormang) correctness + LDS attribution after; dummy-step ablation (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3l; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_physics.py tests/test_gpu_edge.py tests/test_gpu_parity_long.py -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for lib in libtgsim.so libtgsim_dk0_9.so libtgsim_dk0_18.so libtgsim_dk1_9.so libtgsim_dk1_18.so; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task ThormangWalk --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${lib}_$rep.log 2>&1 || exit $?
    echo "$rep $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${lib}_$rep.log)"
  done
done
OUT_DIR=$OUT/ldsattr TASKS=ThormangWalk timeout -k 10 600 bash scripts/dev/lds_attrib.sh > $OUT/ldsattr.log 2>&1 || exit $?
python3 scripts/dev/lds_attrib.py $OUT/ldsattr ThormangWalk

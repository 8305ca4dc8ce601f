# scooters on lane pairs with 16-byte env strides: parity + every bench config (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3y; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gogoro.py tests/test_gpu_paper.py tests/test_gpu_terrain.py tests/test_gpu_physics.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for a in "Gogoro 4096" "GogoroPaper 4096" "GogoroPaper 2048" "ThormangWalk 4096"; do
  set -- $a
  timeout -k 10 200 python bench.py --task $1 --num-envs $2 --steps 500 --warmup 50 --no-cpu-baseline > $OUT/bench_$1_$2.log 2>&1 || exit $?
  echo "$1 $2 $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_$1_$2.log | tr '\n' ' ')"
done
timeout -k 10 200 python bench.py --task Gogoro --num-envs 4096 --steps 500 --warmup 50 --terrain --no-cpu-baseline > $OUT/bench_terrain.log 2>&1 || exit $?
echo "terrain $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_terrain.log | tr '\n' ' ')"

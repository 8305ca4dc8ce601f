#!/bin/bash
# Round-2 closing evidence (last session): the full GPU test suite, the bench
# line of every workload in DESIGN.md §5, the driver's distributed launch form
# at one rank, and rocprofv3 kernel statistics of the three step paths.  Every
# GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final2
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_default.log | cut -c1-200
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$n.log 2>&1
  local rc=$?; echo "bench $n rc=$rc $(tail -c 2000 $OUT/bench_$n.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
run thormangwalkdr4096 --task ThormangWalkDR --no-cpu-baseline
run thormangwalk8192 --task ThormangWalk --num-envs 8192 --no-cpu-baseline
run thormangwalk16384 --task ThormangWalk --num-envs 16384 --no-cpu-baseline
run thormangwalkdr16384 --task ThormangWalkDR --num-envs 16384 --no-cpu-baseline
run gogoro4096 --task Gogoro
run gogoro4096_terrain --task Gogoro --terrain
run gogoropaper2048 --task GogoroPaper --num-envs 2048 --no-cpu-baseline
run gogoropaper4096 --task GogoroPaper --no-cpu-baseline
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 200 --warmup 50 --no-cpu-baseline > $OUT/bench_torchrun_n1.log 2>&1 || exit $?
tail -1 $OUT/bench_torchrun_n1.log | cut -c1-200
for t in ThormangWalk Gogoro GogoroPaper; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_$t -o run -- python3 bench.py --task $t --steps 300 --warmup 50 --no-cpu-baseline > $OUT/trace_$t.log 2>&1 || exit $?
  cut -d, -f1-4 $OUT/trace_$t/run_kernel_stats.csv | head -3
done
exit 0

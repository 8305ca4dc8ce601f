#!/bin/bash
# Round-2 closing evidence on one MI355X: the full GPU test suite, the default
# bench line (N=1, with the CPU baseline) and the driver's distributed launch
# form at one rank (torchrun + RCCL barrier / max-over-ranks reduction).
# Every GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_default.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 200 --warmup 50 --no-cpu-baseline > $OUT/bench_torchrun_n1.log 2>&1 || exit $?
tail -1 $OUT/bench_torchrun_n1.log | cut -c1-300
exit 0

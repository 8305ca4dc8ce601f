#!/bin/bash
# Iteration loop on the GPU box: selected parity tests (PYTEST_K), then a
# short bench of each workload in BENCH_TASKS.  Every GPU step has its own
# time limit and a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-walk or physics}" > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
for t in ${BENCH_TASKS:-ThormangWalk}; do
  timeout -k 10 200 python bench.py --task $t --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline > gpurun_out/iter_bench_$t.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $t rc=$rc"; tail -5 gpurun_out/iter_bench_$t.log; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/iter_bench_$t.log').read().strip().splitlines()[-1]); print('$t', '%.4g'%d['value'], 'kernel_ms %.4f'%d['roofline']['kernel_ms'])"
done

#!/bin/bash
# Quick iteration session: the named GPU tests, then the ThormangWalk and
# Gogoro bench lines and a rocprofv3 kernel-trace summary of each.  Every GPU
# step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/quick}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" $OUT/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
fi
for t in ${TASKS:-ThormangWalk Gogoro}; do
  timeout -k 10 300 python bench.py --task $t --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline > $OUT/bench_$t.log 2>&1 || exit $?
  echo "$t $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_$t.log | tr '\n' ' ')"
  if [ -n "${PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_$t -o run -- python3 bench.py --task $t --steps 200 --warmup 30 --no-cpu-baseline > $OUT/trace_$t.log 2>&1 || exit $?
    cut -d, -f1-4 $OUT/trace_$t/run_kernel_stats.csv | head -5
  fi
done
exit 0

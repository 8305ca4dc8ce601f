#!/bin/bash
# Round-4 session: the GPU test suite (optional), named dev scripts, bench
# lines.  Every GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/r4}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; [ $rc -le 1 ] || exit $rc
fi
for spec in ${DEV:-}; do   # script.py[:args-with-commas]
  s=${spec%%:*}; a=""; [ "$s" != "$spec" ] && a=${spec#*:} && a=${a//,/ }
  log=$OUT/$(basename $s .py)$(echo "$a" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40).log
  timeout -k 10 900 python -u $s $a > $log 2>&1 || { echo "$s failed"; tail -20 $log; exit 1; }
  tail -${DEV_TAIL:-5} $log | cut -c1-600
done
for spec in ${BENCHES:-}; do   # name:args-with-commas
  n=${spec%%:*}; a=${spec#*:}; a=${a//,/ }
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$n.log 2>&1 || { echo "bench $n failed"; tail -5 $OUT/bench_$n.log; exit 1; }
  echo "bench $n $(tail -c 3000 $OUT/bench_$n.log | grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
done
exit 0

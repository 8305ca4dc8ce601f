#!/bin/bash
# Round-3 session: GPU tests, the Gogoro drift study with its developer
# builds, the bench lines.  Each GPU step under its own time limit; a step
# that crashes, aborts or times out (rc > 1) ends the script, a test failure
# (rc 1) does not stop the measurements after it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/r3}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ok() { [ "$1" -le 1 ] || { echo "step rc=$1: stopping"; exit "$1"; }; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" $OUT/tests.log | tail -12; ok $rc
fi
if [ -n "${DRIFT:-}" ]; then
  timeout -k 10 900 python -u scripts/parity_drift.py $DRIFT --out $OUT ${VARIANTS:+--variants $VARIANTS} > $OUT/drift_$DRIFT.log 2>&1
  rc=$?; echo "drift rc=$rc"; tail -4 $OUT/drift_$DRIFT.log; ok $rc
fi
for t in ${TASKS:-ThormangWalk Gogoro}; do
  timeout -k 10 300 python bench.py --task $t --steps ${STEPS:-1000} --warmup 100 ${CPU:---no-cpu-baseline} > $OUT/bench_$t.log 2>&1
  rc=$?; ok $rc
  echo "$t $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_$t.log | tr '\n' ' ')"
  if [ -n "${PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_$t -o run -- python3 bench.py --task $t --steps 200 --warmup 30 --no-cpu-baseline > $OUT/trace_$t.log 2>&1
    rc=$?; ok $rc
    cut -d, -f1-4 $OUT/trace_$t/run_kernel_stats.csv | head -4
  fi
done
# in-kernel section profile (s_memtime stamps) of a developer build
if [ -n "${SECT:-}" ]; then
  for t in ${TASKS:-ThormangWalk Gogoro}; do
    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_prof.so timeout -k 10 300 python scripts/section_prof.py $t > $OUT/section_$t.txt 2>&1
    rc=$?; ok $rc; grep -v Warning $OUT/section_$t.txt | grep -v "^ *sp = " | head -16
  done
fi
# A/B: the bench lines again with developer builds (AB="label=path.so ...")
for ab in ${AB:-}; do
  for t in ${TASKS:-ThormangWalk Gogoro}; do
    TG_LIB_PATH=${ab#*=} timeout -k 10 300 python bench.py --task $t --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_${ab%%=*}.log 2>&1
    rc=$?; ok $rc
    echo "$t [${ab%%=*}] $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_${ab%%=*}.log | tr '\n' ' ')"
  done
done
exit 0

#!/bin/bash
# The GPU test suite on its own (one process, per-test time limit), log to
# $OUT/gpu_tests.log; optional pytest -k filter in $K.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/tests}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | tail -n 200 > $OUT/summary.txt || true
tail -3 $OUT/gpu_tests.log
exit $rc

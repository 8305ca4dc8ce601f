#!/bin/bash
# Parity evidence session: the free-running divergence study of every
# workload (scripts/parity_drift.py: GPU vs fp64 oracle, fp64 oracle vs a
# 1e-6-perturbed copy, fp32 oracle build vs fp64), then the long parity
# tests.  Every GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT_DIR:-gpurun_out/drift}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for w in ${DRIFT_WORKLOADS:-gogoro gogoro_fixbase walk walk_stand walk_fixbase}; do
  n=64; case $w in walk*) n=32;; esac
  timeout -k 10 300 python scripts/parity_drift.py $w --steps 1000 --envs $n --out $OUT > $OUT/log_$w.txt 2>&1
  rc=$?; echo "drift $w rc=$rc"; tail -3 $OUT/log_$w.txt; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${PYTEST_FILES:-}" ]; then
  timeout -k 10 900 python -u -m pytest $PYTEST_FILES -m gpu -v --timeout 300 --timeout-method thread -rA > $OUT/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20; exit $rc
fi
exit 0

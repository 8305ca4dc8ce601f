#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Every GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
stop_if_fatal() {  # $1 = exit code, $2 = step name
  if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then
    echo "FATAL: $2 exited $1 -- stopping"; exit "$1"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -q -rA ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -30 gpurun_out/gpu_tests.log; stop_if_fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 200 --warmup 30} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; stop_if_fatal $rc bench
exit 0

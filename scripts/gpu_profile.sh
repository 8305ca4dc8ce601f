#!/bin/bash
# rocprofv3 kernel-trace statistics of the bench workload, then PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate runs, no tracing domains combined).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 200 --warmup 30} --no-cpu-baseline"
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 gpurun_out/prof/trace.log; stop_if_fatal $rc trace
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/prof/pmc_$c -o run -- python3 bench.py $ARGS > gpurun_out/prof/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; tail -2 gpurun_out/prof/pmc_$c.log; stop_if_fatal $rc pmc_$c
done
find gpurun_out/prof -name "*.csv" | head -20
exit 0

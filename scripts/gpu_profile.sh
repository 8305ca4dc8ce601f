#!/bin/bash
# rocprofv3 kernel-trace statistics of the bench workload, then PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate runs, no tracing domains combined).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF=${PROF_DIR:-gpurun_out/prof}
mkdir -p $PROF
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 200 --warmup 30} --no-cpu-baseline"
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PROF/trace -o run -- python3 bench.py $ARGS > $PROF/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 $PROF/trace.log; stop_if_fatal $rc trace
# counter passes: ';'-separated sets, counters within a set share one pass
PMC_SETS="${PMC_SETS:-FETCH_SIZE;WRITE_SIZE}"
IFS=';' read -ra SETS <<< "$PMC_SETS"
for set in "${SETS[@]}"; do
  tag=$(echo $set | awk '{print $1}')
  timeout -k 10 600 rocprofv3 --pmc $set -T --output-format csv -d $PROF/pmc_$tag -o run -- python3 bench.py $ARGS > $PROF/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $set rc=$rc"; tail -2 $PROF/pmc_$tag.log; stop_if_fatal $rc pmc_$tag
done
find $PROF -name "*.csv" | head -20
exit 0

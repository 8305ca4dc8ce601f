#!/bin/bash
# A/B of library builds (developer): bench.py per task with each library
# (TG_LIB_PATH), ROUNDS interleaved rounds, one line per run with the
# env-steps/s and the step kernel's event-timed ms.
# usage: LIBS="base=thormang_isaacgym_amd/libtgsim.so x=...so" TASKS="ThormangWalk Gogoro" \
#        OUT=gpurun_out/ab scripts/dev/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/ab}
ROUNDS=${ROUNDS:-2}
TASKS=${TASKS:-ThormangWalk Gogoro}
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for t in $TASKS; do
    for kv in $LIBS; do
      n=${kv%%=*}; p=${kv#*=}
      TG_LIB_PATH=$p timeout -k 10 200 python bench.py --task $t --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${t}_${n}_$r.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || { echo "$t $n rc=$rc"; tail -5 $OUT/${t}_${n}_$r.log; exit $rc; }
      echo "$t $n r$r $(tail -c 4000 $OUT/${t}_${n}_$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
    done
  done
done | tee $OUT/summary.txt

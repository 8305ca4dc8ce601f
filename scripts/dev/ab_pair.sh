#!/bin/bash
# Developer A/B of two libraries: bit comparison over 100 steps of every task
# (scripts/dev/bitcmp_libs.py), then bench.py for each task in $TASKS, two
# interleaved rounds.  A = libtgsim.so (the product), B = $B (a variant in
# thormang_isaacgym_amd/).  Output under $OUT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/ab}
B=${B:?variant library name}
TASKS=${TASKS:-ThormangWalk Gogoro}
mkdir -p $OUT
L=thormang_isaacgym_amd
if [ -z "${NO_BITCMP:-}" ]; then
timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/a.npz > $OUT/bit_a.log 2>&1 || { tail -5 $OUT/bit_a.log; exit 1; }
TG_LIB_PATH=$L/$B timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/b.npz > $OUT/bit_b.log 2>&1 || { tail -5 $OUT/bit_b.log; exit 1; }
python scripts/dev/bitcmp_libs.py cmp $OUT/b.npz $OUT/a.npz | tee $OUT/bitcmp.txt
fi
for r in 1 2; do
  for task in $TASKS; do
    for v in A:libtgsim.so B:$B; do
      n=${v%%:*}; lib=${v#*:}
      TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task $task --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${task}_${n}_r$r.log 2>&1 \
        || { echo "$task $n failed"; tail -5 $OUT/${task}_${n}_r$r.log; exit 1; }
      echo "$task $n($lib) r$r $(tail -c 4000 $OUT/${task}_${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
    done
  done
done | tee $OUT/summary.txt

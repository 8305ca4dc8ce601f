#!/bin/bash
# Round 5 (developer): the cost of honouring sim.physx.contact_offset (VERDICT
# r4 item 4): each task's cfg value against --contact-offset 0 (every point
# within contact_margin carries a row, the round-4 behaviour), same library,
# two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/coff}
mkdir -p $OUT
for r in 1 2; do
  for task in ThormangWalk Gogoro; do
    for v in cfg:"" off:"--contact-offset 0"; do
      n=${v%%:*}; opt=${v#*:}
      timeout -k 10 200 python bench.py --task $task --no-cpu-baseline $opt > $OUT/${task}_${n}_r$r.log 2>&1 \
        || { echo "$task $n failed"; tail -5 $OUT/${task}_${n}_r$r.log; exit 1; }
      echo "$task $n r$r $(tail -c 4000 $OUT/${task}_${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
    done
  done
done | tee $OUT/summary.txt

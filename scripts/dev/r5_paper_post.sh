#!/bin/bash
# Round 5 (developer): GogoroPaper 4096, where the post launch's time goes --
# the product (term-7 batch sum and the push-force reduction inside the post
# launch) against the finish launch (TG_PAPER_FINISH=1) and the separate
# rb_force_kernel launch (TG_PAPER_RB_LAUNCH=1), rocprof kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/paperpost}
mkdir -p $OUT
export TMPDIR=/tmp
for v in product: finish:TG_PAPER_FINISH=1 rblaunch:TG_PAPER_RB_LAUNCH=1; do
  n=${v%%:*}; e=${v#*:}
  if [ -n "$e" ]; then export "$e"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 bench.py --task GogoroPaper --steps 300 --warmup 50 --no-cpu-baseline > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  unset TG_PAPER_FINISH TG_PAPER_RB_LAUNCH
  echo "== $n $(grep -o '"value": [0-9.e+]*' $OUT/$n.log | head -1)"
  f=$(find $OUT/$n -name '*kernel_stats.csv' | head -1)
  head -6 "$f" | cut -d, -f1-4
done | tee $OUT/summary.txt

#!/bin/bash
# Round 5 (developer): what the tree passes' parent / child LDS traffic costs
# the headline walk step -- TG_PROBE builds (results wrong) in which pass 1a
# (1), pass 2b (2), pass 3 (4), the impulse top-down pass (8) or all (15) take
# the parent's / child's values from the lane's own previous-step registers
# instead of LDS, against the product library; two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/probe}
mkdir -p $OUT
L=thormang_isaacgym_amd
for r in 1 2; do
  for v in base:libtgsim.so p1:libtgsim_probe1.so p2:libtgsim_probe2.so p4:libtgsim_probe4.so \
           p8:libtgsim_probe8.so p15:libtgsim_probe15.so; do
    n=${v%%:*}; lib=${v#*:}
    TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task ThormangWalk --no-cpu-baseline \
      > $OUT/${n}_r$r.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_r$r.log; exit 1; }
    echo "$n r$r $(tail -c 4000 $OUT/${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
  done
done | tee $OUT/summary.txt

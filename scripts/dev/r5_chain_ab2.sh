#!/bin/bash
# Round 5 (developer): the chain schedule's default (TG_CHAIN_MASK 7: passes
# 1a, 2b and 3) against the list schedule (bit-for-bit over 100 steps of every
# task, scripts/dev/bitcmp_libs.py) and its speed beside the list schedule and
# the all-passes form (mask 15, the impulse pass too), ThormangWalk, two
# interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/chain2}
mkdir -p $OUT
L=thormang_isaacgym_amd
timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/chain.npz > $OUT/bit_chain.log 2>&1 || { tail -5 $OUT/bit_chain.log; exit 1; }
TG_LIB_PATH=$L/libtgsim_list.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/list.npz > $OUT/bit_list.log 2>&1 || { tail -5 $OUT/bit_list.log; exit 1; }
python scripts/dev/bitcmp_libs.py cmp $OUT/chain.npz $OUT/list.npz | tee $OUT/bitcmp.txt
for r in 1 2; do
  for v in chain7:libtgsim.so list:libtgsim_list.so chain15:libtgsim_cm15.so; do
    n=${v%%:*}; lib=${v#*:}
    TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task ThormangWalk --no-cpu-baseline > $OUT/${n}_r$r.log 2>&1 \
      || { echo "$n failed"; tail -5 $OUT/${n}_r$r.log; exit 1; }
    echo "ThormangWalk $n r$r $(tail -c 4000 $OUT/${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
  done
done | tee $OUT/summary.txt

#!/bin/bash
# Round 5 (developer): the impulse pass in chain form with every lane storing
# the joint velocities (TG_CHAIN_MASK 15, the product default) against the
# list schedule, bit for bit over 100 steps of every task, and its speed beside
# mask 7 (the impulse pass in list form), the list schedule and the build
# without the forwarded-value laundering, ThormangWalk, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/chain15}
mkdir -p $OUT
L=thormang_isaacgym_amd
timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/main.npz > $OUT/bit_main.log 2>&1 || { tail -5 $OUT/bit_main.log; exit 1; }
TG_LIB_PATH=$L/libtgsim_list.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/list.npz > $OUT/bit_list.log 2>&1 || { tail -5 $OUT/bit_list.log; exit 1; }
TG_LIB_PATH=$L/libtgsim_nol.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/nol.npz > $OUT/bit_nol.log 2>&1 || { tail -5 $OUT/bit_nol.log; exit 1; }
{ echo "== main (mask 15) vs list"; python scripts/dev/bitcmp_libs.py cmp $OUT/main.npz $OUT/list.npz;
  echo "== no-launder vs list"; python scripts/dev/bitcmp_libs.py cmp $OUT/nol.npz $OUT/list.npz; } | tee $OUT/bitcmp.txt
for r in 1 2; do
  for v in chain15:libtgsim.so chain7:libtgsim_cm7.so list:libtgsim_list.so nolaunder:libtgsim_nol.so; do
    n=${v%%:*}; lib=${v#*:}
    TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task ThormangWalk --no-cpu-baseline > $OUT/${n}_r$r.log 2>&1 \
      || { echo "$n failed"; tail -5 $OUT/${n}_r$r.log; exit 1; }
    echo "ThormangWalk $n r$r $(tail -c 4000 $OUT/${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
  done
done | tee $OUT/summary.txt

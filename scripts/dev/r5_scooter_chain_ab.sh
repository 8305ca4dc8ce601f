#!/bin/bash
# Round 5 (developer): the chain schedule on the scooters' 6-group trees
# (TG_CHAIN_MIN_NG=2, libtgsim_chs.so) against the product (list schedule for
# them): bit comparison over 100 steps of every task, then Gogoro and
# GogoroPaper 4096, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/scooter_chain}
mkdir -p $OUT
L=thormang_isaacgym_amd
timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/main.npz > $OUT/bit_main.log 2>&1 || { tail -5 $OUT/bit_main.log; exit 1; }
TG_LIB_PATH=$L/libtgsim_chs.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/chs.npz > $OUT/bit_chs.log 2>&1 || { tail -5 $OUT/bit_chs.log; exit 1; }
python scripts/dev/bitcmp_libs.py cmp $OUT/chs.npz $OUT/main.npz | tee $OUT/bitcmp.txt
for r in 1 2; do
  for task in Gogoro GogoroPaper; do
    for v in main:libtgsim.so chs:libtgsim_chs.so; do
      n=${v%%:*}; lib=${v#*:}
      TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task $task --no-cpu-baseline > $OUT/${task}_${n}_r$r.log 2>&1 \
        || { echo "$task $n failed"; tail -5 $OUT/${task}_${n}_r$r.log; exit 1; }
      echo "$task $n r$r $(tail -c 4000 $OUT/${task}_${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
    done
  done
done | tee $OUT/summary.txt

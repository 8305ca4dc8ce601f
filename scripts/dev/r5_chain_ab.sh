#!/bin/bash
# Round 5 (developer): the chain schedule (TG_CHAIN=1, the product library)
# against the list schedule (libtgsim_list.so, TG_CHAIN=0): bit-for-bit
# comparison of 100 steps of every task (scripts/dev/bitcmp_libs.py), then
# the walk and Gogoro bench lines, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/chain}
mkdir -p $OUT
L=thormang_isaacgym_amd
timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/chain.npz > $OUT/bit_chain.log 2>&1 || { tail -5 $OUT/bit_chain.log; exit 1; }
TG_LIB_PATH=$L/libtgsim_list.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/list.npz > $OUT/bit_list.log 2>&1 || { tail -5 $OUT/bit_list.log; exit 1; }
python scripts/dev/bitcmp_libs.py cmp $OUT/chain.npz $OUT/list.npz | tee $OUT/bitcmp.txt
if [ -f $L/libtgsim_nosync.so ]; then
  TG_LIB_PATH=$L/libtgsim_nosync.so timeout -k 10 300 python scripts/dev/bitcmp_libs.py run $OUT/nosync.npz > $OUT/bit_nosync.log 2>&1 || { tail -5 $OUT/bit_nosync.log; exit 1; }
  python scripts/dev/bitcmp_libs.py cmp $OUT/nosync.npz $OUT/list.npz | tee $OUT/bitcmp_nosync.txt
fi
for r in 1 2; do
  for t in ThormangWalk Gogoro; do
    for v in chain:libtgsim.so list:libtgsim_list.so nosync:libtgsim_nosync.so; do
      n=${v%%:*}; lib=${v#*:}
      TG_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --task $t --no-cpu-baseline > $OUT/${t}_${n}_r$r.log 2>&1 \
        || { echo "$t $n failed"; tail -5 $OUT/${t}_${n}_r$r.log; exit 1; }
      echo "$t $n r$r $(tail -c 4000 $OUT/${t}_${n}_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
    done
  done
done | tee $OUT/summary.txt

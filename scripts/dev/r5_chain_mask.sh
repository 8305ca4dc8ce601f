#!/bin/bash
# Round 5 (developer): which tree pass's chain form changes the rounding --
# the per-step states of a 12-step walk run (scripts/dev/step_states.py) of the
# list schedule against builds with the chain registers in one pass only
# (TG_CHAIN_MASK 1, 2, 4, 8) and in all (the product library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/chainmask}
mkdir -p $OUT
L=thormang_isaacgym_amd
TG_LIB_PATH=$L/libtgsim_list.so timeout -k 10 200 python scripts/dev/step_states.py run $OUT/list.npz || exit 1
for v in ${VARIANTS:-cm1 cm2 cm4 cm8}; do
  TG_LIB_PATH=$L/libtgsim_$v.so timeout -k 10 200 python scripts/dev/step_states.py run $OUT/$v.npz || exit 1
  echo "== $v vs list"; python scripts/dev/step_states.py cmp $OUT/$v.npz $OUT/list.npz | head -4
done | tee $OUT/summary.txt

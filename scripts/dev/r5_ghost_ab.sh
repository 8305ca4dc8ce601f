#!/bin/bash
# Round 5, VERDICT r4 item 1 prototype A/B (developer): what a second wave
# per SIMD buys the headline walk.  Libraries (scripts/dev builds):
#   base     the product kernel: 4096 envs = 1024 waves, 1 per SIMD, 310 registers
#   alias16  the same kernel compiled for 2 waves per SIMD (256 registers, spills)
#            but still 16 envs per workgroup: 1 wave per SIMD -- the spill control
#   ghost    TG_GHOST_DEV: 2 real envs per wave, 2 waves per SIMD (same spills)
#   alias8   TG_ALIAS_DEV=8: 2 workgroups per CU, full waves (results wrong)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/ghost}
mkdir -p $OUT
L=thormang_isaacgym_amd
run() {  # name lib envs
  TG_LIB_PATH=$L/$2 timeout -k 10 200 python bench.py --task ThormangWalk --num-envs $3 --no-cpu-baseline \
    > $OUT/$1_$3_r$r.log 2>&1 || { echo "$1 $3 failed"; tail -5 $OUT/$1_$3_r$r.log; exit 1; }
  echo "$1 envs=$3 r$r $(tail -c 4000 $OUT/$1_$3_r$r.log | grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
}
for r in 1 2; do
  run base libtgsim.so 4096
  run alias16 libtgsim_alias16.so 4096
  run ghost libtgsim_ghost.so 4096
  run base libtgsim.so 8192
  run alias8 libtgsim_alias8.so 8192
  run ghost libtgsim_ghost.so 8192
done | tee $OUT/summary.txt

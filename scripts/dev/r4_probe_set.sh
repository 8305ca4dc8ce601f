#!/bin/bash
# Round-4 probe set (developer): scheduler-unit A/B against the previous
# library (libtgsim_base.so), a bit-for-bit check that the two builds agree,
# the standing walk teacher-forced, the DR-16384 outlier scan and the three
# drift studies.  Output under gpurun_out/d3 and gpurun_out/ab2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/d3
mkdir -p $O
LIBS="base=thormang_isaacgym_amd/libtgsim_base.so new=thormang_isaacgym_amd/libtgsim.so" \
  TASKS="ThormangWalk Gogoro GogoroPaper ThormangWalkDR" OUT=gpurun_out/ab2 bash scripts/dev/ab_libs.sh || exit $?
V=thormang_isaacgym_amd/libtgsim_v_
LIBS="new=thormang_isaacgym_amd/libtgsim.so minreg=${V}minreg.so maxocc=${V}maxocc.so topdown=${V}topdown.so bidir=${V}bidir.so nounclust=${V}nounclust.so postbu=${V}postbu.so postbi=${V}postbi.so trk=${V}trk.so" \
  TASKS="ThormangWalk Gogoro" OUT=gpurun_out/ab3 bash scripts/dev/ab_libs.sh || exit $?
TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_base.so timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_base.npz > $O/bc_base.log 2>&1 || exit $?
timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_new.npz > $O/bc_new.log 2>&1 || exit $?
python scripts/dev/bitcmp_libs.py cmp $O/bc_base.npz $O/bc_new.npz > $O/bitcmp.txt
timeout -k 10 300 python -u scripts/dev/standing_forced.py 32 1000 21 > $O/standing_forced.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/dev/forced_outliers.py ThormangWalkDR 16384 100 12 > $O/outliers.log 2>&1 || exit $?
for w in "walk_stand 32" "walk 64" "gogoro 64"; do
  set -- $w
  timeout -k 10 300 python -u scripts/parity_drift.py $1 --steps 1000 --envs $2 --seed 21 --out $O > $O/drift_$1.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tests.gpu_harness import walk_env_vs_oracle
print(walk_env_vs_oracle(num_envs=32, steps=1000, seed=21, amp=0.0, control=True))" > $O/standing_free.txt 2>&1

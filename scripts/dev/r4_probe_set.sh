#!/bin/bash
# Round-4 probe set (developer), most important first: a bit-for-bit check
# that the scheduler-split library agrees with the previous one
# (libtgsim_base.so), the standing walk test, the A/B of the two libraries,
# the scheduler sweep, the standing walk teacher-forced, the DR-16384 outlier
# scan and the three drift studies.  Output under gpurun_out/d3, ab2, ab3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/d3
mkdir -p $O
TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_base.so timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_base.npz > $O/bc_base.log 2>&1 || exit $?
timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_new.npz > $O/bc_new.log 2>&1 || exit $?
python scripts/dev/bitcmp_libs.py cmp $O/bc_base.npz $O/bc_new.npz > $O/bitcmp.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_long.py -k standing -s -q --timeout 380 --timeout-method thread > $O/standing_test.txt 2>&1
LIBS="base=thormang_isaacgym_amd/libtgsim_base.so new=thormang_isaacgym_amd/libtgsim.so" \
  TASKS="ThormangWalk Gogoro GogoroPaper ThormangWalkDR" OUT=gpurun_out/ab2 bash scripts/dev/ab_libs.sh || exit $?
V=thormang_isaacgym_amd/libtgsim_v_
LIBS="new=thormang_isaacgym_amd/libtgsim.so minreg=${V}minreg.so maxocc=${V}maxocc.so topdown=${V}topdown.so bidir=${V}bidir.so nounclust=${V}nounclust.so postbu=${V}postbu.so postbi=${V}postbi.so trk=${V}trk.so" \
  TASKS="ThormangWalk Gogoro" OUT=gpurun_out/ab3 bash scripts/dev/ab_libs.sh || exit $?
timeout -k 10 300 python -u scripts/dev/standing_forced.py 32 1000 21 > $O/standing_forced.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/dev/forced_outliers.py ThormangWalkDR 16384 100 12 > $O/outliers.log 2>&1 || exit $?
for w in "walk_stand 32" "walk 64" "gogoro 64"; do
  set -- $w
  timeout -k 10 300 python -u scripts/parity_drift.py $1 --steps 1000 --envs $2 --seed 21 --out $O > $O/drift_$1.log 2>&1 || exit $?
done

#!/bin/bash
# Round-4 A/B (developer): the row-parallel contact setup (libtgsim.so)
# against one lane per shape (libtgsim_base.so, -DTG_ROW_PAR=0): bit-for-bit
# check, the GPU suite on the new library, then bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/rp
mkdir -p $O
TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_base.so timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_base.npz > $O/bc_base.log 2>&1 || exit $?
timeout -k 10 200 python scripts/dev/bitcmp_libs.py run $O/bc_new.npz > $O/bc_new.log 2>&1 || exit $?
python scripts/dev/bitcmp_libs.py cmp $O/bc_base.npz $O/bc_new.npz > $O/bitcmp.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -le 1 ] || exit $rc
LIBS="base=thormang_isaacgym_amd/libtgsim_base.so new=thormang_isaacgym_amd/libtgsim.so" \
  TASKS="ThormangWalk Gogoro GogoroPaper ThormangWalkDR" OUT=gpurun_out/ab4 bash scripts/dev/ab_libs.sh || exit $?

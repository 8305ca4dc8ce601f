#!/bin/bash
# LDS bank-conflict attribution (developer tool): one rocprofv3 --pmc pass per
# stop-point build (TG_EXTRA_FLAGS=-DTG_STOP_AT=k, libtgsim_stop<k>.so: the
# step kernel returns at its k-th section stamp) and one for the full kernel;
# successive differences give each section's LDS instructions, active cycles
# and bank-conflict cycles (scripts/dev/lds_attrib.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT_DIR:-gpurun_out/ldsattr}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
CTR=${CTR:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"}
for task in ${TASKS:-ThormangWalk Gogoro}; do
  for k in ${STOPS:-0 16 1 17 18 2 3 4 5 6 7 8 full}; do
    lib=thormang_isaacgym_amd/libtgsim_stop$k.so
    [ "$k" = full ] && lib=thormang_isaacgym_amd/libtgsim.so
    d=$OUT/${task}_$k
    TG_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $CTR -T --output-format csv -d $d/pmc_0 -o run \
      -- python3 bench.py --task $task --steps 20 --warmup 5 --no-cpu-baseline > $d.log 2>&1
    rc=$?; echo "$task stop $k rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
    python3 scripts/pmc_summary.py $d > $d.json
  done
done
exit 0

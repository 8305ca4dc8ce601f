#!/bin/bash
# LDS / issue counters of the bench workload (one rocprofv3 --pmc pass per set,
# each under its own time limit; no tracing domains combined with --pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF=${PROF_DIR:-gpurun_out/pmclds}
mkdir -p $PROF
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 100 --warmup 20} --no-cpu-baseline"
SETS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM"
)
i=0
for set in "${SETS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d $PROF/pmc_$i -o run -- python3 bench.py $ARGS > $PROF/pmc_$i.log 2>&1
  rc=$?; echo "pmc set $i rc=$rc"; tail -2 $PROF/pmc_$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
python3 scripts/pmc_summary.py $PROF > $PROF/summary.json
exit 0

# per-section issue / wait counters of the step kernel (stop-point builds; developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3p; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
  OUT_DIR=$OUT/wait timeout -k 10 900 bash scripts/dev/lds_attrib.sh > $OUT/wait.log 2>&1 || { tail -5 $OUT/wait.log; exit 1; }
python3 scripts/dev/lds_attrib.py $OUT/wait

set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3d; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in libtgsim libtgsim_quat libtgsim_pgsr libtgsim_allp; do
  TG_LIB_PATH=thormang_isaacgym_amd/$v.so timeout -k 10 300 python -u scripts/dev/forced_errors.py --label $v >> $OUT/forced.jsonl 2> $OUT/forced_$v.err
  rc=$?; echo "$v rc=$rc"; tail -1 $OUT/forced.jsonl; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 900 python -u scripts/parity_drift.py gogoro --out $OUT --variants quat=thormang_isaacgym_amd/libtgsim_quat.so,allp=thormang_isaacgym_amd/libtgsim_allp.so > $OUT/drift_gogoro.log 2>&1
rc=$?; echo "drift rc=$rc"; cat $OUT/drift_gogoro.txt

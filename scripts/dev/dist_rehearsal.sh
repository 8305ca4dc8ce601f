# developer rehearsal of bench.py's N > 1 path on a one-GPU box: two torchrun
# ranks, gloo for the barrier / max-over-ranks timing reduction, both ranks'
# envs on cuda:0 (RCCL refuses two ranks on one device).  Not a scaling
# number: the two ranks share the one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/dist}; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TG_BENCH_DIST_BACKEND=gloo TG_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 200 --warmup 20 \
  --no-cpu-baseline > $OUT/bench_rehearsal_n2.log 2>&1 || exit $?
grep '^{"metric"' $OUT/bench_rehearsal_n2.log | cut -c1-300
grep -o '"dist": {[^}]*}' $OUT/bench_rehearsal_n2.log

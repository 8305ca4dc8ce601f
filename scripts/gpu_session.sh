#!/bin/bash
# Closing evidence of a round on one MI355X (replaces the per-round
# gpu_final_r2/r2b/r3/r4.sh and gpu_r2_prof/r3/r4.sh scripts): the full GPU
# test suite, smoke(), the bench line of every workload in DESIGN.md §5 (the
# default line with its cpu_baseline), the driver's short form and its
# distributed launch at one rank, rocprofv3 kernel statistics of the three
# step paths, the HBM PMC passes and the SQ / LDS counter passes of the two
# headline workloads, and the register / scratch use of every step kernel.
# Every GPU step has its own time limit; a failure stops the script.
#   ROUND=6 bash scripts/gpu_session.sh            (everything, into gpurun_out/final$ROUND)
#   SKIP_TESTS=1 SKIP_PROF=1 ... / ONLY_PROF=1     (parts; the GPU call's time limit is 20 min)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-6}
OUT=${OUT_DIR:-gpurun_out/final$ROUND}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${ONLY_PROF:-}" ]; then SKIP_TESTS=1; SKIP_BENCH=1; fi
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
  tail -1 $OUT/smoke.log
fi
if [ -z "${SKIP_BENCH:-}" ]; then
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_default.log | cut -c1-300
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$n.log 2>&1
  local rc=$?; echo "bench $n rc=$rc $(tail -c 3000 $OUT/bench_$n.log | grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
run thormangwalk4096_pgs --task ThormangWalk --solver-type 0 --no-cpu-baseline
run thormangwalk4096_wholebody --task ThormangWalk --whole-body --no-cpu-baseline
run thormangwalkdr4096 --task ThormangWalkDR --no-cpu-baseline
run thormangwalk8192 --task ThormangWalk --num-envs 8192 --no-cpu-baseline
run thormangwalk16384 --task ThormangWalk --num-envs 16384 --no-cpu-baseline
run thormangwalkdr16384 --task ThormangWalkDR --num-envs 16384 --no-cpu-baseline
run gogoro4096 --task Gogoro
run gogoro4096_terrain --task Gogoro --terrain --no-cpu-baseline
run gogoropaper2048 --task GogoroPaper --num-envs 2048 --no-cpu-baseline
run gogoropaper4096 --task GogoroPaper --no-cpu-baseline
run driver_form --steps 20 --warmup 5 --no-cpu-baseline
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 200 --warmup 50 --no-cpu-baseline > $OUT/bench_torchrun_n1.log 2>&1 || exit $?
tail -1 $OUT/bench_torchrun_n1.log | cut -c1-200
fi
[ -n "${SKIP_PROF:-}" ] && exit 0
for t in ThormangWalk Gogoro GogoroPaper; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_$t -o run -- python3 bench.py --task $t --steps 300 --warmup 50 --no-cpu-baseline > $OUT/trace_$t.log 2>&1 || exit $?
  cut -d, -f1-4 $OUT/trace_$t/run_kernel_stats.csv | head -3
done
for t in ThormangWalk Gogoro; do
  PROF_DIR=$OUT/hbm_$t BENCH_ARGS="--task $t --steps 200 --warmup 30" timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/hbm_$t.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py $OUT/hbm_$t > $OUT/pmc_$t.json
  PROF_DIR=$OUT/sq_$t BENCH_ARGS="--task $t --steps 100 --warmup 20" timeout -k 10 600 bash scripts/gpu_pmc_lds.sh > $OUT/sq_$t.log 2>&1 || exit $?
  cp $OUT/sq_$t/summary.json $OUT/sq_$t.json
  python3 - $OUT/pmc_$t.json $OUT/sq_$t.json <<'PY'
import json, sys
p = json.load(open(sys.argv[1])); q = json.load(open(sys.argv[2]))
for k, v in p.items():
    if "step_par_kernel" in k: print("hbm bytes/launch", v.get("hbm_bytes_per_dispatch"))
for k, v in q.items():
    if "step_par_kernel" in k:
        a = v["avg"]; print("valu frac %.3f wait frac %.3f lds conflict frac %.3f" % (
            a["SQ_ACTIVE_INST_VALU"] / a["SQ_WAVE_CYCLES"], a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"],
            a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"]))
PY
done
exit 0

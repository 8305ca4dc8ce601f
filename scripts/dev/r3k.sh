# env-stride A/B (developer session): ES = 2 mod 4 variants (TG_ES_PAD) vs the
# current layout -- bench twice each, alternating, then one LDS counter pass each
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3k; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
LIBS=${LIBS:-"libtgsim.so libtgsim_pad2.so libtgsim_pad6.so libtgsim_pad10.so libtgsim_pad14.so"}
for rep in 1 2; do
  for t in ThormangWalk Gogoro; do
    for lib in $LIBS; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_${t}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep $t $lib $(grep -o '"kernel_ms": [0-9.e+]*' $OUT/bench_${t}_${lib}_$rep.log)"
    done
  done
done
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for t in ThormangWalk Gogoro; do
  for lib in $LIBS; do
    d=$OUT/lds_${t}_$lib
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $CTR -T --output-format csv -d $d/pmc_0 -o run \
      -- python3 bench.py --task $t --steps 20 --warmup 5 --no-cpu-baseline > $d.log 2>&1 || exit $?
    python3 scripts/pmc_summary.py $d > $d.json
    python3 -c "import json; e=json.load(open('$d.json'))['step_par_kernel']['avg']; print('$t $lib', 'LDS instr/wave %.0f' % (e['SQ_INSTS_LDS']/e['SQ_WAVES']), 'conflict frac %.3f' % (e['SQ_LDS_BANK_CONFLICT']/e['SQ_LDS_IDX_ACTIVE']))"
  done
done

# what two waves per SIMD would buy: LDS-aliased envs (wrong results, timing only) compiled for 2 waves/SIMD (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3s; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for n in 4096 8192 16384; do
    for lib in libtgsim.so libtgsim_alias8.so; do
      TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task ThormangWalk --num-envs $n --steps 500 --warmup 50 --no-cpu-baseline > $OUT/bench_${n}_${lib}_$rep.log 2>&1 || exit $?
      echo "$rep N=$n $lib $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $OUT/bench_${n}_${lib}_$rep.log | tr '\n' ' ')"
    done
  done
done

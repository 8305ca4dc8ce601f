set -u
mkdir -p gpurun_out
for lib in libtgsim.so libtgsim_hot.so; do
  TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/ab_$lib.log 2>&1 || exit $?
  echo "$lib $(python -c "import json; d=json.loads(open('gpurun_out/ab_$lib.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])")"
done

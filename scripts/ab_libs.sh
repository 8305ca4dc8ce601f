# developer A/B: bench tasks (TASKS) with each library named on the command line
# (thormang_isaacgym_amd/<lib>), one GPU step each
set -u
mkdir -p gpurun_out
for t in ${TASKS:-ThormangWalk Gogoro}; do
  for lib in "$@"; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 200 python bench.py --task $t --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
    echo "$t $lib $(python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('%.4g'%d['value'], '%.4f'%d['roofline']['kernel_ms'])")"
  done
done

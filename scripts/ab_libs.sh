# developer A/B: bench a task under different env settings (one GPU step each)
set -u
mkdir -p gpurun_out
t=${TASK:-Gogoro}
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --task $t --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
  echo "$t [$cfg] $(python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])")"
done

#!/bin/bash
# rocprofv3 kernel stats of scripts/dev/paper_compose_variants.py, one run per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in fused unfused nopush; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pcv/$v -o run -- python3 scripts/dev/paper_compose_variants.py $v > gpurun_out/pcv_$v.log 2>&1 || exit $?
  echo "== $v"; cut -d, -f1-4 gpurun_out/pcv/$v/run_kernel_stats.csv | head -7
done

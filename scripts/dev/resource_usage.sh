#!/bin/bash
# Register / scratch / LDS use of every step_par_kernel instantiation
# (hipcc -Rpass-analysis=kernel-resource-usage on articulation.hip).
# usage: EXTRA="extra hipcc flags" scripts/dev/resource_usage.sh
set -eu
REPO=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${TMPDIR:-/tmp}/tg_ru
mkdir -p $OUT
# the two units, each with its machine scheduler (build_ext.py)
: > $OUT/ru.txt
for u in "articulation.hip max-ilp" "articulation_tree.hip iterative-ilp"; do
  set -- $u
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -ffast-math -fno-associative-math -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics -fno-slp-vectorize -mllvm --amdgpu-sched-strategy=$2 ${EXTRA:-} \
    -Rpass-analysis=kernel-resource-usage -c $REPO/thormang_isaacgym_amd/csrc/$1 -o $OUT/a.o 2>> $OUT/ru.txt
done
python3 - $OUT/ru.txt <<'PY'
import re, subprocess, sys
txt = open(sys.argv[1]).read()
print("VGPR AGPR scratch occ LDS  kernel")
for b in txt.split("Function Name: ")[1:]:
    name = b.split("\n")[0]
    if "step_par_kernel" not in name:
        continue
    g = lambda k: (re.search(k + r": (\d+)", b) or [None, "?"])[1]
    dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip().replace("tg::", "")
    dn = re.sub(r"void step_par_kernel<", "<", dn)[:100]
    print(g("VGPRs"), g("AGPRs"), g(r"ScratchSize \[bytes/lane\]"), g(r"Occupancy \[waves/SIMD\]"),
          g(r"LDS Size \[bytes/block\]"), dn)
PY

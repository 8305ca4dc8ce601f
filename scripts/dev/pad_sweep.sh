#!/bin/bash
# Developer experiment: step-kernel time vs the LDS env-stride padding
# (libtgsim_padN.so built with TG_EXTRA_FLAGS=-DTG_ES_PAD=N).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pad
for lib in libtgsim.so libtgsim_pad4.so libtgsim_pad8.so libtgsim_pad12.so libtgsim_pad16.so libtgsim_pad20.so libtgsim_pad24.so libtgsim_pad28.so; do
  for t in ThormangWalk Gogoro; do
    TG_LIB_PATH=thormang_isaacgym_amd/$lib timeout -k 10 120 python bench.py --task $t --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/pad/$lib.$t.log 2>&1 || exit $?
    echo "$lib $t $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' gpurun_out/pad/$lib.$t.log | tr '\n' ' ')"
  done
done

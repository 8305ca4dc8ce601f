"""Build libtgsim.so in-tree for gfx950 (hipcc; cross-compiles without a GPU).

Steps: regenerate the constexpr model traits (model/codegen.py), compile the
three translation units with their own numerics flags, link a shared library
next to this file.  Incremental: a unit is rebuilt only when a source or
header it depends on is newer than its object."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(REPO, "build", "tgsim")
LIB = os.path.join(HERE, os.environ.get("TG_LIB_NAME", "libtgsim.so"))
# developer builds (e.g. TG_EXTRA_FLAGS=-DTG_SECTION_PROF TG_LIB_NAME=libtgsim_prof.so) get their own objects
EXTRA = os.environ.get("TG_EXTRA_FLAGS", "").split()
if EXTRA:
    BUILD = BUILD + "_" + "_".join(f.strip("-").replace("=", "_") for f in EXTRA)
ARCH = os.environ.get("TG_OFFLOAD_ARCH", "gfx950")


def _sched(env, dflt):
    """-mllvm scheduler flags of a unit (developer override: TG_SCHED_MAIN /
    TG_SCHED_TREE = a strategy name, 'default', or raw -mllvm options after
    'raw:' separated by commas)"""
    v = os.environ.get(env, dflt)
    if v == "default":
        return []
    if v.startswith("raw:"):
        return [x for o in v[4:].split(",") if o for x in ("-mllvm", o)]
    return ["-mllvm", f"--amdgpu-sched-strategy={v}"]


SCHED_MAIN = _sched("TG_SCHED_MAIN", "max-ilp")
SCHED_TREE = _sched("TG_SCHED_TREE", "iterative-ilp")
for _k in ("TG_SCHED_MAIN", "TG_SCHED_TREE"):   # developer variants get their own objects
    if _k in os.environ:
        BUILD = BUILD + "_" + _k[-4:].lower() + "_" + "".join(c if c.isalnum() else "_" for c in os.environ[_k])
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

UNITS = {
    # physics: fast-math lets zero tree terms fold away in the specialised kernels
    # (SLP pairing into v_pk_* costs more register moves than it saves here:
    # Gogoro step 0.226 -> 0.128 ms without it, Thormang unchanged)
    # -ffp-contract=fast-honor-pragmas after -ffast-math: contraction stays on
    # for the physics, but the fused task epilogues' `#pragma clang fp
    # contract(off)` blocks (the reference's fp32 operation order) are honoured
    # -- plain -ffast-math lets the backend fuse a*b+c there regardless
    # -fno-associative-math (round 4): reassociated sums rounded the GPU 2-6x
    # further from the fp64 oracle than its fp32 build in the rounding-
    # sensitive runs (GogoroPaper reward 2.0e-3 -> 7.1e-4, 8192-env walk
    # reward 1.2e-3 -> 7.1e-4, teacher-forced) for +1.4 % step time; the
    # other fast-math parts (reciprocals, approximate functions) measured
    # no parity effect (DESIGN.md §2 "GPU rounding")
    # The step kernels are split over two units by tree size (launch.h
    # in_unit) so that each gets the machine scheduler that measured fastest
    # for it (round 4, scripts/dev/ab_libs.sh): the scooters
    # and the known-answer models the max-ILP strategy, the humanoid trees
    # the iterative ILP one.  Scheduling reorders instructions only; the
    # arithmetic, and with it every result, is the same
    "articulation.hip": ["-O3", "-ffast-math", "-fno-associative-math", "-ffp-contract=fast-honor-pragmas",
                         "-munsafe-fp-atomics", "-fno-slp-vectorize", *SCHED_MAIN],
    "articulation_tree.hip": ["-O3", "-ffast-math", "-fno-associative-math", "-ffp-contract=fast-honor-pragmas",
                              "-munsafe-fp-atomics", "-fno-slp-vectorize", *SCHED_TREE],
    # task math must follow the reference's fp32 operation order
    "gogoro_task.hip": ["-O3", "-ffp-contract=off"],
    "walk_task.hip": ["-O3", "-ffp-contract=off"],
    "gogoro_paper_task.hip": ["-O3", "-ffp-contract=off"],
    "tgsim_api.cpp": ["-O2", "-x", "hip"],
    # run-time specialisations (hipRTC) of the articulation kernels
    "jit.cpp": ["-O2", "-x", "hip"],
    # native URDF loading (tg_model_parse / tg_model_load): host C++ only
    "model_load.cpp": ["-O2"],
}


def _deps():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "generated", "*.inc"))
            + glob.glob(os.path.join(REPO, "include", "*.h")))


def build(verbose: bool = False, jobs: int = 4) -> str:
    sys.path.insert(0, REPO)
    from thormang_isaacgym_amd.model import codegen
    codegen.generate(os.path.join(CSRC, "generated"))
    os.makedirs(BUILD, exist_ok=True)
    dep_mtime = max(os.path.getmtime(p) for p in _deps())
    procs, objs = [], []
    for src, flags in UNITS.items():
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src + ".o")
        objs.append(o)
        if os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), dep_mtime):
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
               "-Wno-unused-variable", *flags, *EXTRA, "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{out.decode(errors='replace')[-6000:]}")
        if verbose and out:
            print(out.decode(errors="replace")[-3000:])
    if procs or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB, "-lhiprtc", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))

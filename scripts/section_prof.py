"""Per-section cycle breakdown of the LDS articulation kernel (developer tool).

Needs the profiling build:
    TG_EXTRA_FLAGS=-DTG_SECTION_PROF TG_LIB_NAME=libtgsim_prof.so python thormang_isaacgym_amd/build_ext.py
    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_prof.so python scripts/section_prof.py
Add -DTG_CLAMP_COUNT to also count the drive-clamp reruns (ThormangWalk: 0 %,
Gogoro: 40 % of env-substeps; the counters' atomics then inflate pass 1).
"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import thormang_isaacgym_amd as tia  # noqa: E402
from thormang_isaacgym_amd import _lib  # noqa: E402

NAMES = ["load", "pass1", "pass2", "pass3", "contact setup", "delassus", "pgs", "apply", "integrate", "store"]


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "ThormangWalk"
    env = tia.make(seed=0, task=task, num_envs=4096, sim_device="cuda:0", rl_device="cuda:0")
    L = _lib.lib()
    L.tg_prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(20):
        env.step(torch.rand(4096, env.num_actions, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 24)()
    L.tg_prof_read(buf, 24)
    # sub-sections [16..] are cut out of the section that follows them
    if os.environ.get("TG_PROF_RAW"):
        print("raw slots:", list(buf))
    sec = list(buf[:len(NAMES)])
    sec[1] += buf[16] + buf[20]
    sec[2] += buf[17] + buf[18]
    tot = sum(sec)
    subs = {1: [("1a schedule fwd", 16), ("1a, substep 0 (TG_PROF_SPLIT0)", 20), ("1b all groups", None)],
            2: [("2a all groups", 17), ("2b schedule bwd", 18), ("root solve", None)]}
    for i, (n, v) in enumerate(zip(NAMES, sec)):
        print(f"{n:14s} {v / tot * 100:6.2f} %  {v:14d}")
        for sn, k in subs.get(i, []):
            sv = buf[k] if k is not None else buf[i]
            print(f"   {sn:16s} {sv / tot * 100:6.2f} %")
    L.tg_cprof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    cb = (C.c_ulonglong * 8)()
    L.tg_cprof_read(cb, 8)
    ctot = sum(cb[:4])
    if ctot:
        print("compose_kernel (cycles summed over composed envs):")
        for n, v in zip(["loads + local joint", "level FK + link mass", "group sums + cache rows", "shapes"], cb):
            print(f"  {n:26s} {v / ctot * 100:6.2f} %  {v:14d}")
    if buf[12]:
        print(f"drive-clamp rerun: {buf[13] / buf[12] * 100:.1f} % of env-substeps, "
              f"{buf[15] / max(buf[14], 1) * 100:.1f} % of wavefront-substeps")


if __name__ == "__main__":
    main()

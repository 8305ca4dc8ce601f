"""Developer probe (GPU, TG_DUMP_ENV build): one env-step of the teacher-forced
16384-env ThormangWalkDR run (scripts/dev/r6_walk_dr_probe.py) -- the
kernel's and the fp64 oracle's contact solve of env ENV at step STEP, per
substep, from identical inputs.

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_dump.so \
        python scripts/dev/r6_walk_dump.py step env [torch_seed] [num_envs]
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import (NumpyDraws, OracleWalk, make_gpu_walk, sync_dr, sync_oracle_from_gpu,  # noqa: E402
                               walk_cfg)
from thormang_isaacgym_amd._lib import lib as tglib  # noqa: E402

STEP, ENV = int(sys.argv[1]), int(sys.argv[2])
tseed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n = int(sys.argv[4]) if len(sys.argv) > 4 else 16384
seed = 12
G = tglib()
G.tg_debug_dump_env.argtypes = [C.c_int, C.c_int]
G.tg_debug_dump_read.argtypes = [C.c_void_p, C.c_int]
np.set_printoptions(precision=6, suppress=True, linewidth=230)


def run(sub):
    mk = lambda: walk_cfg(n, "ThormangWalkDR", dr=True)
    env = make_gpu_walk(mk(), NumpyDraws(seed), torch_seed=tseed)
    orc = OracleWalk(mk(), NumpyDraws(seed))
    orc.L.oracle_dump_set.argtypes = [C.c_int, C.c_int]
    orc.L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
    rs = np.random.default_rng(seed + 100)
    for t in range(STEP + 1):
        sync_oracle_from_gpu(orc, env)
        sync_dr(orc, env)
        act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
        if t == STEP:
            G.tg_debug_dump_env(ENV, sub)
            orc.L.oracle_dump_set(ENV, sub)
            root0 = env.root_tensor[ENV].cpu().numpy().copy()
        env.step(torch.from_numpy(act).to("cuda:0"))
        orc.step(act)
    torch.cuda.synchronize()
    g = np.zeros(4096, np.float32)
    G.tg_debug_dump_read(g.ctypes.data, 4096)
    o = np.zeros(4096, np.float64)
    orc.L.oracle_dump_read(o.ctypes.data, 4096)
    G.tg_debug_dump_env(-1, 0)
    orc.L.oracle_dump_set(-1, 0)
    return g, o, env.root_tensor[ENV].cpu().numpy(), orc.a["root"][ENV].copy(), root0, orc.D


for sub in range(2):
    g, o, rg, ro, root0, D = run(sub)
    K = int(o[0]) if o[0] else int(g[0])
    print(f"--- step {STEP} env {ENV} substep {sub}: K gpu {int(g[0])} oracle {int(o[0])}")
    if sub == 0:
        print("  root before", root0)
        print("  root after gpu   ", rg)
        print("  root after oracle", ro)
    for name, off, m in (("a0", 2700, 6), ("v0", 2710, 6), ("qdd", 2800, D), ("vfree", 2000, K),
                         ("lam_pos", 2600, K), ("lam_vel", 2500, K)):
        a, b = g[off:off + m], o[off:off + m]
        k = int(np.argmax(np.abs(a - b)))
        print(f"  {name}: max|gpu-o| {np.abs(a - b).max():.2e} at {k} (|o| max {np.abs(b).max():.3g})")
        if name in ("lam_pos", "lam_vel", "vfree", "a0"):
            print("     gpu   ", a)
            print("     oracle", b)
    print("  phi/targets gpu   ", g[2100 + 6:2100 + 8 * K:8])
    print("  phi/targets oracle", o[2100 + 6:2100 + 8 * K:8])
    Wg, Wo = g[16:16 + K * K].reshape(K, K), o[16:16 + K * K].reshape(K, K)
    d = np.abs(Wg - Wo)
    i, j = np.unravel_index(np.argmax(d), d.shape)
    print(f"  W: max|gpu-o| {d.max():.2e} at ({i},{j}) (|W| max {np.abs(Wo).max():.3g}); clamp flag gpu {g[2790]} "
          f"oracle {o[2790]}")

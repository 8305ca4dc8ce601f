"""Developer probe (GPU, TG_DUMP_ENV build): the Gogoro 4096-env teacher-
forced outlier (scripts/dev/gogoro_forced_outliers.py: seed 23, the bench's
U(-1,1) actions) -- one env's dynamics and contact solve in each substep of
one step, kernel beside the fp64 oracle from identical inputs.

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_dump.so \
        python scripts/dev/gogoro_contact_dump.py [step] [env] [num_envs] [seed]
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, make_gpu_gogoro, parity_cfg, sync_oracle_from_gpu  # noqa
from thormang_isaacgym_amd._lib import lib as tglib  # noqa: E402

STEP = int(sys.argv[1]) if len(sys.argv) > 1 else -1    # -1: pass 1 finds the worst (step, env)
ENV = int(sys.argv[2]) if len(sys.argv) > 2 else -1
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 23
SCAN = int(sys.argv[5]) if len(sys.argv) > 5 else 100
G = tglib()
G.tg_debug_dump_env.argtypes = [C.c_int, C.c_int]
G.tg_debug_dump_read.argtypes = [C.c_void_p, C.c_int]


def find_worst():
    env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
    orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
    rs = np.random.default_rng(n)
    worst = (0.0, -1, -1, -1)
    for t in range(SCAN):
        sync_oracle_from_gpu(orc, env)
        act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
        od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
        o_obs = orc.step(act[:, 0])[0]
        e = np.abs(od["obs"].cpu().numpy() - o_obs)
        i = int(np.argmax(e.max(1)))
        if e[i].max() > worst[0]:
            worst = (float(e[i].max()), t, i, int(np.argmax(e[i])))
    return worst


if STEP < 0:
    w = find_worst()
    print("pass 1: largest teacher-forced obs error %.2e at step %d env %d (component %d)" % w)
    STEP, ENV = w[1], w[2]


def run(sub):
    env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
    orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
    orc.L.oracle_dump_set.argtypes = [C.c_int, C.c_int]
    orc.L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
    rs = np.random.default_rng(n)
    for t in range(STEP + 1):
        sync_oracle_from_gpu(orc, env)
        act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
        if t == STEP:
            G.tg_debug_dump_env(ENV, sub)
            orc.L.oracle_dump_set(ENV, sub)
            root0 = orc.a["root"][ENV].copy()
        od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
        o_obs = orc.step(act[:, 0])[0].copy()
    torch.cuda.synchronize()
    g = np.zeros(4096, np.float32)
    G.tg_debug_dump_read(g.ctypes.data, 4096)
    o = np.zeros(4096, np.float64)
    orc.L.oracle_dump_read(o.ctypes.data, 4096)
    G.tg_debug_dump_env(-1, 0)   # (disarm: also clears the dump buffers)
    orc.L.oracle_dump_set(-1, 0)
    return g, o, od["obs"][ENV].cpu().numpy(), o_obs[ENV], root0, orc.D


np.set_printoptions(precision=7, suppress=True, linewidth=220)
out = {}
for sub in range(3):
    g, o, og, oo, root0, D = run(sub)
    out[f"gpu{sub}"], out[f"oracle{sub}"] = g, o
    K = int(o[0]) if o[0] else int(g[0])
    print(f"--- step {STEP} env {ENV} substep {sub}: K {K}; obs gpu {og} oracle {oo}")
    if sub == 0:
        print("    root before the step", root0)
    for name, off, m in (("a0", 2700, 6), ("v0", 2710, 6), ("qdd", 2800, D), ("vfree", 2000, K),
                         ("lam_pos", 2600, K), ("lam_vel", 2500, K)):
        a, b = g[off:off + m], o[off:off + m]
        k = int(np.argmax(np.abs(a - b)))
        print(f"{name}: max|gpu-o| {np.abs(a - b).max():.2e} at {k} (|o| max {np.abs(b).max():.3g})")
        if name in ("lam_pos", "lam_vel", "a0", "vfree"):
            print("   gpu   ", a)
            print("   oracle", b)
    pg, po = g[2100 + 6:2100 + 8 * K:8], o[2100 + 6:2100 + 8 * K:8]
    print("phi/targets gpu   ", pg)
    print("phi/targets oracle", po)
    Wg, Wo = g[16:16 + K * K].reshape(K, K), o[16:16 + K * K].reshape(K, K)
    print(f"W: max|gpu-o| {np.abs(Wg - Wo).max():.2e} (|W| max {np.abs(Wo).max():.3g}); drive clamp flag {g[2790]}")
np.savez("gpurun_out/gogoro_contact_dump.npz", **out)

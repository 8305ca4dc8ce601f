"""Developer probe (GPU, TG_DUMP_ENV build): one env's contact solve in the
kernel and in the fp64 oracle from identical inputs -- the Delassus matrix W,
the free row velocities and the multipliers -- at the step where the
teacher-forced walk run's largest GPU-only error sits
(scripts/dev/forced_outliers.py: ThormangWalk 8192 envs seed 11, step 98,
env 7631).

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_dump.so python scripts/dev/contact_dump.py [step] [env]
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_oracle_from_gpu, walk_cfg  # noqa: E402
from thormang_isaacgym_amd._lib import lib as tglib  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 98
E = int(sys.argv[2]) if len(sys.argv) > 2 else 7631
n, seed, task = 8192, 11, "ThormangWalk"
env = make_gpu_walk(walk_cfg(n, task), NumpyDraws(seed))
orc = OracleWalk(walk_cfg(n, task), NumpyDraws(seed))
ctl = OracleWalk(walk_cfg(n, task), NumpyDraws(seed), precision="f32")
rs = np.random.default_rng(seed + 100)
G = tglib()
G.tg_debug_dump_env.argtypes = [C.c_int]
G.tg_debug_dump_read.argtypes = [C.c_void_p, C.c_int]
for L in (orc.L, ctl.L):
    L.oracle_dump_set.argtypes = [C.c_int]
    L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
for t in range(T + 1):
    sync_oracle_from_gpu(orc, env)
    sync_oracle_from_gpu(ctl, env)
    act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
    last = t == T
    G.tg_debug_dump_env(E if last else -1)
    orc.L.oracle_dump_set(E if last else -1)
    ctl.L.oracle_dump_set(E if last else -1)
    od, rew, _, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    o_obs, o_rew = [x.copy() for x in orc.step(act)[:2]]
    c_obs, c_rew = [x.copy() for x in ctl.step(act)[:2]]
g = np.zeros(4096, np.float32)
G.tg_debug_dump_read(g.ctypes.data, 4096)
o = np.zeros(4096, np.float64)
orc.L.oracle_dump_read(o.ctypes.data, 4096)
c = np.zeros(4096, np.float64)
ctl.L.oracle_dump_read(c.ctypes.data, 4096)
K = int(o[0])
print("K gpu", int(g[0]), "oracle", K, "env", E, "step", T)
np.set_printoptions(precision=6, suppress=True, linewidth=220)
Wg, Wo, Wc = (x[16:16 + K * K].reshape(K, K) for x in (g, o, c))
rel = lambda a, b: np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
print("W: max|gpu-o| %.2e (rel %.2e)  max|f32-o| %.2e  asym gpu %.2e o %.2e" % (
    np.abs(Wg - Wo).max(), rel(Wg, Wo), np.abs(Wc - Wo).max(), np.abs(Wg - Wg.T).max(), np.abs(Wo - Wo.T).max()))
i, j = np.unravel_index(np.argmax(np.abs(Wg - Wo)), Wg.shape)
print("   worst W entry", (i, j), "gpu", Wg[i, j], "oracle", Wo[i, j], "f32", Wc[i, j])
for name, off in (("vfree", 2000), ("lam_vel", 2500), ("lam_pos", 2600)):
    a, b, cc = g[off:off + K], o[off:off + K], c[off:off + K]
    print(f"{name}: max|gpu-o| {np.abs(a - b).max():.2e}  max|f32-o| {np.abs(cc - b).max():.2e}")
    print("   gpu   ", a)
    print("   oracle", b)
    print("   f32   ", cc)
for name, off, m in (("a0", 2700, 6), ("v0", 2710, 6), ("qdd", 2800, orc.D)):
    a, b, cc = g[off:off + m], o[off:off + m], c[off:off + m]
    k = int(np.argmax(np.abs(a - b)))
    print(f"{name}: max|gpu-o| {np.abs(a - b).max():.2e} at {k}  max|f32-o| {np.abs(cc - b).max():.2e}")
    print("   gpu   ", a[:12])
    print("   oracle", b[:12])
print("gpu drive-clamp flag", g[2790])
print("obs[4:7] gpu", od["obs"][E, 4:7].cpu().numpy(), "oracle", o_obs[E, 4:7], "f32", c_obs[E, 4:7])

"""Developer probe (GPU, TG_DUMP_ENV build): one env's dynamics and contact
solve in the kernel and in the fp64 oracle from identical inputs -- the root
free acceleration, the joint accelerations, the Delassus matrix W, the free
row velocities and the multipliers -- in each substep of the step where the
teacher-forced walk run's largest base yaw-rate error sits.  Pass 1 finds
that (step, env) under this build; pass 2 replays to it and dumps.

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_dump.so python scripts/dev/contact_dump.py [steps]
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_oracle_from_gpu, walk_cfg  # noqa: E402
from thormang_isaacgym_amd._lib import lib as tglib  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 100
n, seed, task = 8192, 11, "ThormangWalk"
G = tglib()
G.tg_debug_dump_env.argtypes = [C.c_int, C.c_int]
G.tg_debug_dump_read.argtypes = [C.c_void_p, C.c_int]


def run(stop=None, env_dump=-1):
    env = make_gpu_walk(walk_cfg(n, task), NumpyDraws(seed))
    orc = OracleWalk(walk_cfg(n, task), NumpyDraws(seed))
    rs = np.random.default_rng(seed + 100)
    orc.L.oracle_dump_set.argtypes = [C.c_int, C.c_int]
    orc.L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
    worst = (0.0, -1, -1)
    dumps = []
    for t in range(STEPS if stop is None else stop + 1):
        sync_oracle_from_gpu(orc, env)
        act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
        if stop is not None and t == stop:
            # the dumped step, once per substep (the oracle re-synced each time)
            state = {k: v.copy() for k, v in orc.a.items()}
            gstate = [x.clone() for x in (env.sim.root_state, env.sim.dof_state)]
            for sub in range(2):
                for k, v in state.items():
                    orc.a[k][...] = v
                env.sim.root_state.copy_(gstate[0])
                env.sim.dof_state.copy_(gstate[1])
                G.tg_debug_dump_env(env_dump, sub)
                orc.L.oracle_dump_set(env_dump, sub)
                od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
                o_obs = orc.step(act)[0].copy()
                g = np.zeros(4096, np.float32)
                G.tg_debug_dump_read(g.ctypes.data, 4096)
                o = np.zeros(4096, np.float64)
                orc.L.oracle_dump_read(o.ctypes.data, 4096)
                dumps.append((g, o, od["obs"][env_dump].cpu().numpy(), o_obs[env_dump]))
            return dumps, orc.D
        od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
        o_obs = orc.step(act)[0]
        e6 = np.abs(od["obs"][:, 6].cpu().numpy() - o_obs[:, 6])
        i = int(np.argmax(e6))
        if e6[i] > worst[0]:
            worst = (float(e6[i]), t, i)
    return worst, None


worst, _ = run()
print("pass 1: largest base yaw-rate obs error %.2e at step %d env %d" % worst)
dumps, D = run(stop=worst[1], env_dump=worst[2])
np.savez("gpurun_out/contact_dump.npz", **{f"{side}{sub}": d[k] for sub, d in enumerate(dumps)
                                          for k, side in ((0, "gpu"), (1, "oracle"))})
np.set_printoptions(precision=6, suppress=True, linewidth=220)
for sub, (g, o, og, oo) in enumerate(dumps):
    K = int(o[0]) if o[0] else int(g[0])
    print(f"--- substep {sub}: K {K}, obs[4:7] gpu {og[4:7]} oracle {oo[4:7]}")
    for name, off, m in (("a0", 2700, 6), ("v0", 2710, 6), ("qdd", 2800, D), ("vfree", 2000, K),
                         ("lam_pos", 2600, K), ("lam_vel", 2500, K)):
        a, b = g[off:off + m], o[off:off + m]
        k = int(np.argmax(np.abs(a - b)))
        print(f"{name}: max|gpu-o| {np.abs(a - b).max():.2e} at {k} (|o| max {np.abs(b).max():.3g})")
        if name.startswith("lam") or name == "a0":
            print("   gpu   ", a)
            print("   oracle", b)
    pg, po = g[2100 + 6:2100 + 8 * K:8], o[2100 + 6:2100 + 8 * K:8]
    print(f"phi (normal rows): max|gpu-o| {np.abs(pg - po).max():.2e}")
    print("   gpu   ", pg)
    print("   oracle", po)
    Wg, Wo = g[16:16 + K * K].reshape(K, K), o[16:16 + K * K].reshape(K, K)
    print(f"W: max|gpu-o| {np.abs(Wg - Wo).max():.2e} (|W| max {np.abs(Wo).max():.3g})")

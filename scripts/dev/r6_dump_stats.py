"""Developer study (GPU, TG_DUMP_ENV build), VERDICT r5 item 1: WHERE in a
substep the scooter's GPU-only rounding excess arises.  Teacher-forced Gogoro
(the bench's batch and actions); at every step one random env's substep-0
intermediates are dumped by the kernel, the fp64 oracle and its fp32 build
from identical inputs (root acceleration a0 and velocity v0 of the free
dynamics, joint accelerations qdd, the Delassus matrix W, free row
velocities vfree, the multipliers), and the GPU's and the fp32 build's error
against fp64 are compared per intermediate over all samples (median / q90 of
the per-sample max error, and their ratio).  The intermediate where the
ratio first rises above ~1 is where the excess is made.

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_dump.so python scripts/dev/r6_dump_stats.py [envs] [steps] [seed] [sub]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, make_gpu_gogoro, parity_cfg, sync_oracle_from_gpu  # noqa
from thormang_isaacgym_amd._lib import lib as tglib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 23
SUB = int(sys.argv[4]) if len(sys.argv) > 4 else 0
G = tglib()
G.tg_debug_dump_env.argtypes = [C.c_int, C.c_int]
G.tg_debug_dump_read.argtypes = [C.c_void_p, C.c_int]
env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
ctl = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16, precision="f32")
for o in (orc, ctl):
    o.L.oracle_dump_set.argtypes = [C.c_int, C.c_int]
    o.L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
D = orc.D
rs = np.random.default_rng(n)
pick = np.random.default_rng(seed + 7)
FIELDS = (("a0", 2700, 6), ("v0", 2710, 6), ("qdd", 2800, D), ("vfree", 2000, None), ("W", 16, None),
          ("lam_pos", 2600, None), ("lam_vel", 2500, None))
eg = {f[0]: [] for f in FIELDS}
ec = {f[0]: [] for f in FIELDS}
og, oc = [], []
skipped = 0
for t in range(steps):
    sync_oracle_from_gpu(orc, env)
    sync_oracle_from_gpu(ctl, env)
    e = int(pick.integers(n))
    G.tg_debug_dump_env(e, SUB)
    orc.L.oracle_dump_set(e, SUB)
    ctl.L.oracle_dump_set(e, SUB)
    act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
    od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
    o_obs = orc.step(act[:, 0])[0].copy()
    c_obs = ctl.step(act[:, 0])[0].copy()
    torch.cuda.synchronize()
    g = np.zeros(4096, np.float32)
    G.tg_debug_dump_read(g.ctypes.data, 4096)
    o = np.zeros(4096, np.float64)
    orc.L.oracle_dump_read(o.ctypes.data, 4096)
    c = np.zeros(4096, np.float64)
    ctl.L.oracle_dump_read(c.ctypes.data, 4096)
    G.tg_debug_dump_env(-1, 0)
    orc.L.oracle_dump_set(-1, 0)
    ctl.L.oracle_dump_set(-1, 0)
    K = int(o[0])
    if K <= 0 or int(g[0]) != K or int(c[0]) != K or bool(env.reset_buf[e].item()):
        skipped += 1
        continue
    g_obs = od["obs"][e].cpu().numpy()
    og.append(float(np.abs(g_obs - o_obs[e]).max()))
    oc.append(float(np.abs(c_obs[e] - o_obs[e]).max()))
    for name, off, m in FIELDS:
        m = K * K if name == "W" else (K if m is None else m)
        a, b, r = g[off:off + m].astype(np.float64), o[off:off + m], c[off:off + m]
        sc = max(float(np.abs(b).max()), 1e-30)
        eg[name].append(float(np.abs(a - b).max()) / sc)
        ec[name].append(float(np.abs(r - b).max()) / sc)
lib = os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so"))
print(f"== {lib}: {len(og)} dumped env-steps (substep {SUB}; {skipped} skipped: no contact / K mismatch / reset)")
print("relative error (max over the vector / its max |fp64|): median, q90 -- gpu | f32 | ratio")
for name, *_ in FIELDS + (("obs(abs)",),):
    a, b = (np.array(og), np.array(oc)) if name == "obs(abs)" else (np.array(eg[name]), np.array(ec[name]))
    qa, qb = np.quantile(a, [0.5, 0.9]), np.quantile(b, [0.5, 0.9])
    print(f"  {name:9s} gpu {qa[0]:.2e} {qa[1]:.2e} | f32 {qb[0]:.2e} {qb[1]:.2e} | ratio "
          f"{qa[0] / max(qb[0], 1e-30):.2f} {qa[1] / max(qb[1], 1e-30):.2f}", flush=True)

"""Developer probe (GPU): where the largest one-step errors of a teacher-forced
Gogoro run sit at the headline batch (4096 envs, the bench's U(-1,1)
actions) -- per step the GPU's worst env and obs component, the fp32 oracle
build's error at that env, and the GPU's and the fp32 build's per-env error
binned by the env origin's distance from the world origin (a GPU-only error
that grows with it is world-coordinate rounding).

    python scripts/dev/gogoro_forced_outliers.py [num_envs] [steps] [seed]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, make_gpu_gogoro, parity_cfg, sync_oracle_from_gpu  # noqa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 23
env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
ctl = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16, precision="f32")
rs = np.random.default_rng(n)
org = np.linalg.norm(env.root_tensor[:, 0:2].cpu().numpy(), axis=1)
rows, eg_env, ec_env = [], np.zeros(n), np.zeros(n)
comp_g, comp_c = np.zeros(6), np.zeros(6)
for t in range(steps):
    sync_oracle_from_gpu(orc, env)
    sync_oracle_from_gpu(ctl, env)
    act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
    od, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    o_obs, o_rew = [x.copy() for x in orc.step(act[:, 0])[:2]]
    c_obs, c_rew = [x.copy() for x in ctl.step(act[:, 0])[:2]]
    g_obs, g_rew = od["obs"].cpu().numpy(), rew.cpu().numpy()
    eg, ec = np.abs(g_obs - o_obs), np.abs(c_obs - o_obs)
    eg_env = np.maximum(eg_env, eg.max(1))
    ec_env = np.maximum(ec_env, ec.max(1))
    comp_g = np.maximum(comp_g, eg.max(0))
    comp_c = np.maximum(comp_c, ec.max(0))
    i = int(np.argmax(eg.max(1)))
    rows.append((float(eg[i].max()), t, i, int(np.argmax(eg[i])), float(ec[i].max()), float(ec.max()), float(org[i]),
                 float(np.abs(g_rew - o_rew).max()), float(np.abs(c_rew - o_rew).max())))
rows.sort(reverse=True)
print("gpu_obs_err step env comp ctl_err_same_env ctl_err_max origin_dist gpu_rew_err ctl_rew_err")
for r in rows[:12]:
    print("%.2e %4d %5d %d %.2e %.2e %7.1f %.2e %.2e" % r)
np.set_printoptions(precision=3, suppress=False, linewidth=200)
print("per obs component max: gpu", comp_g, "\n                        f32", comp_c)
bins = [0, 16, 32, 64, 96, 128, 1e9]
print("origin distance bin: envs, median/max per-env obs err  gpu | f32")
for lo, hi in zip(bins[:-1], bins[1:]):
    m = (org >= lo) & (org < hi)
    if m.any():
        print("  [%4.0f,%4.0f) %5d  gpu %.2e / %.2e | f32 %.2e / %.2e" % (
            lo, min(hi, 999), m.sum(), np.median(eg_env[m]), eg_env[m].max(), np.median(ec_env[m]), ec_env[m].max()))

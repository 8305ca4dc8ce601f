"""Developer probe (GPU): where the largest one-step errors of a teacher-forced
walk run sit -- per step the GPU's worst env for the reward, the fp32 oracle
build's error at that same env, and the fp32 build's own worst, so a GPU-only
outlier (the fp32 build quiet there) stands apart from a rounding-sensitive
state (both large).

    python scripts/dev/forced_outliers.py [task] [num_envs] [steps] [seed]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_dr, sync_oracle_from_gpu, walk_cfg  # noqa

task = sys.argv[1] if len(sys.argv) > 1 else "ThormangWalkDR"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 12
env = make_gpu_walk(walk_cfg(n, task), NumpyDraws(seed))
orc = OracleWalk(walk_cfg(n, task), NumpyDraws(seed))
ctl = OracleWalk(walk_cfg(n, task), NumpyDraws(seed), precision="f32")
rs = np.random.default_rng(seed + 100)
rows = []
detail = {}
for t in range(steps):
    sync_oracle_from_gpu(orc, env)
    sync_oracle_from_gpu(ctl, env)
    act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
    od, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    o_obs, o_rew = [x.copy() for x in orc.step(act)[:2]]
    c_obs, c_rew = [x.copy() for x in ctl.step(act)[:2]]
    g_rew, g_obs = rew.cpu().numpy(), od["obs"].cpu().numpy()
    eg, ec = np.abs(g_rew - o_rew), np.abs(c_rew - o_rew)
    i = int(np.argmax(eg))
    og = np.abs(g_obs[i] - o_obs[i])
    rows.append((float(eg[i]), t, i, float(ec[i]), float(ec.max()), int(np.argmax(og)), float(og.max()),
                 float(np.abs(c_obs[i] - o_obs[i]).max())))
    detail[t] = dict(env=i, prog=int(orc.a["progress_buf"][i]), reset=int(orc.a["reset_buf"][i]),
                     root_o=orc.a["root"][i].copy(), root_g=env.root_tensor[i].cpu().numpy(),
                     root_c=ctl.a["root"][i].copy(), obs_o=o_obs[i, :13], obs_g=g_obs[i, :13], obs_c=c_obs[i, :13])
rows.sort(reverse=True)
print("gpu_rew_err step env ctl_rew_err_same_env ctl_rew_err_max obs_comp gpu_obs_err ctl_obs_err")
for r in rows[:12]:
    print("%.2e %4d %6d %.2e %.2e %3d %.2e %.2e" % r)
np.set_printoptions(precision=6, suppress=True, linewidth=200)
for r in rows[:3]:
    d = detail[r[1]]
    print(f"step {r[1]} env {d['env']} progress {d['prog']} reset {d['reset']}")
    for k in ("root_o", "root_g", "root_c", "obs_o", "obs_g", "obs_c"):
        print("  ", k, d[k])
eg_all = np.array([r[0] for r in rows])
print("steps with gpu rew err > 1e-3:", int((eg_all > 1e-3).sum()), "of", steps)

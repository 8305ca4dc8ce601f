"""Developer probe (GPU): the standing walk (zero actions: the PD-held default
pose, tests/test_gpu_parity_long.py's standing workload) teacher-forced --
the fp64 oracle and its fp32 build re-synced from the GPU env before every
step -- so the one-step errors of the GPU and of the fp32 build against fp64
are compared on the same states: per step the max over envs and obs
components, summarised over the steps.

    python scripts/dev/standing_forced.py [num_envs] [steps] [seed] [amp]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_dr, sync_oracle_from_gpu, walk_cfg  # noqa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 21
amp = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
env = make_gpu_walk(walk_cfg(n), NumpyDraws(seed))
orc = OracleWalk(walk_cfg(n), NumpyDraws(seed))
ctl = OracleWalk(walk_cfg(n), NumpyDraws(seed), precision="f32")
rs = np.random.default_rng(seed + 100)
g_err, c_err, g_env, c_env = [], [], np.zeros(n), np.zeros(n)
for t in range(steps):
    for o in (orc, ctl):
        sync_oracle_from_gpu(o, env)
        sync_dr(o, env)
    act = (rs.uniform(-amp, amp, (n, orc.D)) if amp > 0 else np.zeros((n, orc.D))).astype(np.float32)
    obs_d = env.step(torch.from_numpy(act).to("cuda:0"))[0]
    o_obs = orc.step(act)[0]
    c_obs = ctl.step(act)[0]
    g = np.abs(obs_d["obs"].cpu().numpy() - o_obs).max(axis=1)
    c = np.abs(c_obs - o_obs).max(axis=1)
    g_err.append(g.max())
    c_err.append(c.max())
    g_env = np.maximum(g_env, g)
    c_env = np.maximum(c_env, c)
g_err, c_err = np.array(g_err), np.array(c_err)
q = lambda x: " ".join(f"{k} {np.percentile(x, p):.2e}" for k, p in (("p50", 50), ("p90", 90), ("p99", 99))) + \
    f" max {x.max():.2e}"
print(f"standing forced: {n} envs x {steps} steps, seed {seed}, amp {amp}")
print("per-step max over envs, GPU vs fp64:     ", q(g_err))
print("per-step max over envs, fp32 vs fp64:    ", q(c_err))
print(f"steps where GPU > fp32 build: {int((g_err > c_err).sum())} of {steps}")
print("per-env max, GPU:                        ", q(g_env))
print("per-env max, fp32 build:                 ", q(c_env))

"""Developer study (GPU), VERDICT r5 item 1: the scooter's per-step rounding
excess.  Teacher-forced Gogoro at the bench's batch and actions: every step
the fp64 oracle and its fp32 build are re-synced from the GPU env, so each
compares one step from identical inputs.  Prints, for the library TG_LIB_PATH
names, the quantiles of |GPU - fp64| and |fp32 - fp64| over all env-steps per
observation component (obs[1] roll rate, obs[2] yaw rate are the body rates),
and their ratio -- a quantile ratio is stable where the max is one outlier.

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_x.so python scripts/dev/r6_gogoro_excess.py [envs] [steps] [seed]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, make_gpu_gogoro, parity_cfg, sync_oracle_from_gpu  # noqa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 23
lib = os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so"))
env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
ctl = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16, precision="f32")
rs = np.random.default_rng(n)
eg, ec, rg, rc = [], [], [], []
for t in range(steps):
    sync_oracle_from_gpu(orc, env)
    sync_oracle_from_gpu(ctl, env)
    act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
    od, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    o_obs, o_rew = [x.copy() for x in orc.step(act[:, 0])[:2]]
    c_obs, c_rew = [x.copy() for x in ctl.step(act[:, 0])[:2]]
    g_obs, g_rew = od["obs"].cpu().numpy(), rew.cpu().numpy()
    eg.append(np.abs(g_obs - o_obs))
    ec.append(np.abs(c_obs - o_obs))
    rg.append(np.abs(g_rew - o_rew))
    rc.append(np.abs(c_rew - o_rew))
eg, ec = np.concatenate(eg), np.concatenate(ec)
rg, rc = np.concatenate(rg), np.concatenate(rc)
qs = (0.5, 0.9, 0.99, 0.999)


def q(x):
    return [float(np.quantile(x, p)) for p in qs] + [float(x.max())]


print(f"== {lib} gogoro teacher-forced {n} envs x {steps} steps seed {seed}: quantiles {qs} + max")
for name, g, c in (("obs1", eg[:, 1], ec[:, 1]), ("obs2", eg[:, 2], ec[:, 2]), ("obs_all", eg.max(1), ec.max(1)),
                   ("rew", rg, rc)):
    a, b = q(g), q(c)
    print(f"{lib:24s} {name:7s} gpu " + " ".join(f"{x:.2e}" for x in a) + " | f32 " + " ".join(f"{x:.2e}" for x in b)
          + " | ratio " + " ".join(f"{x / max(y, 1e-30):.2f}" for x, y in zip(a, b)), flush=True)

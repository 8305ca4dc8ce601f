"""Developer probe (GPU): where the GogoroPaper teacher-forced run's largest
one-step reward / obs errors sit (tests/test_gpu_paper.py's 300-step forced
test, flags flipped: free base), beside the fp32 oracle build's error at the
same (step, env) -- per step the GPU's worst env, its obs component, and the
control's error there.

    python scripts/dev/paper_forced_scan.py [steps]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, sync_dr, sync_oracle_from_gpu  # noqa: E402
from tests.paper_harness import OraclePaper  # noqa: E402
from tests.test_gpu_paper import FLIPPED, switches  # noqa: E402
from thormang_isaacgym_amd.cfg import load_task_cfg  # noqa: E402
from thormang_isaacgym_amd.tasks.gogoro_cfg import env_origins  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
n, seed = 64, 3
cfg = load_task_cfg("GogoroPaper", num_envs=n)
cfg["env"]["max_steps"] = 60
cfg["noises"]["speed_freq_update"] = cfg["noises"]["yaw_freq_update"] = 25
with switches(FLIPPED) as gp:
    class Env(gp.Gogoro):
        draw_source = NumpyDraws(seed)
    env = Env(cfg, "cuda:0", "cuda:0", -1, True, False, False)
    full = dict(gp.current_switches())
mk = lambda prec: OraclePaper(load_task_cfg("GogoroPaper", num_envs=n) | {"env": cfg["env"], "noises": cfg["noises"]},
                              NumpyDraws(seed), full, root_origins=env_origins(n, 1.0), precision=prec)
orc, ctl = mk("f64"), mk("f32")
rs = np.random.default_rng(seed + 7)
rows = []
for t in range(steps):
    for o in (orc, ctl):
        sync_oracle_from_gpu(o, env)
        sync_dr(o, env)
    act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
    od, rew, reset, ex = env.step(torch.from_numpy(act).cuda())
    o_obs, o_rew = orc.step(act[:, 0])[:2]
    c_obs, c_rew = ctl.step(act[:, 0])[:2]
    g_obs, g_rew = od["obs"].cpu().numpy(), rew.cpu().numpy()
    ge = np.abs(g_rew - o_rew)
    ce = np.abs(c_rew - o_rew)
    e = int(ge.argmax())
    oe = np.abs(g_obs[e] - o_obs[e])
    rows.append((float(ge[e]), t, e, float(ce[e]), float(ce.max()), int(oe.argmax()), float(oe.max()),
                 float(np.abs(c_obs[e] - o_obs[e]).max()), float(o_rew[e])))
rows.sort(reverse=True)
print("gpu_rew_err step env ctl_rew_err_same_env ctl_rew_err_max obs_comp gpu_obs_err ctl_obs_err rew")
for r in rows[:15]:
    print("%.2e %4d %4d %.2e %.2e %4d %.2e %.2e %.4f" % r)
g = np.array([r[0] for r in rows])
c = np.array([r[4] for r in rows])
print("per-step max: gpu p50 %.2e p99 %.2e max %.2e | fp32 p50 %.2e p99 %.2e max %.2e" % (
    np.median(g), np.percentile(g, 99), g.max(), np.median(c), np.percentile(c, 99), c.max()))

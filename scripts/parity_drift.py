"""Developer diagnostic: per-component GPU-vs-oracle drift over a long run.

    python scripts/parity_drift.py [Gogoro|ThormangWalk] [steps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.gpu_harness import (NumpyDraws, OracleGogoro, OracleWalk, balance_policy, make_gpu_gogoro,  # noqa: E402
                               make_gpu_walk, parity_cfg, walk_cfg)


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "Gogoro"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    if task == "Gogoro":
        n = 64
        env = make_gpu_gogoro(parity_cfg(n, max_steps=300), NumpyDraws(21))
        orc = OracleGogoro(parity_cfg(n, max_steps=300), NumpyDraws(21))
        obs = orc.a["obs_buf"].copy()
        act_fn = lambda o: balance_policy(o)
    else:
        n = 32
        env = make_gpu_walk(walk_cfg(n), NumpyDraws(7))
        orc = OracleWalk(walk_cfg(n), NumpyDraws(7))
        rs = np.random.default_rng(107)
        act_fn = lambda o: rs.uniform(-0.3, 0.3, (n, orc.D)).astype(np.float32)
        obs = None
    win = np.zeros(0)
    for t in range(steps):
        act = act_fn(obs)
        od, rew, reset, ex = env.step(torch.from_numpy(act).cuda())
        if task == "Gogoro":
            o_obs, o_rew, o_reset, o_to = orc.step(act[:, 0])
        else:
            o_obs, o_rew, o_reset, o_to = orc.step(act)
        g_obs = od["obs"].cpu().numpy()
        d = np.abs(g_obs - o_obs).max(axis=0)
        if d.max() > 1e-3 and not getattr(main, "reported", False):
            main.reported = True
            e = int(np.abs(g_obs - o_obs).max(axis=1).argmax())
            np.set_printoptions(precision=6, suppress=True, linewidth=200)
            print(f"first >1e-3 at step {t}, env {e}")
            print(" gpu obs", g_obs[e][:10])
            print(" orc obs", o_obs[e][:10])
            print(" gpu root", env.root_tensor.cpu().numpy()[e])
            print(" orc root", orc.a["root"][e])
            D = orc.a["dof_state"].shape[0] // n
            gd = env.state_dof.cpu().numpy().reshape(n, D, 2)[e]
            od_ = orc.a["dof_state"].reshape(n, D, 2)[e]
            k = np.abs(gd - od_).max(axis=1)
            top = np.argsort(k)[::-1][:5]
            print(" worst dofs", top.tolist(), k[top])
            print(" gpu dof", gd[top])
            print(" orc dof", od_[top])
        win = d if win.size == 0 else np.maximum(win, d)
        obs = o_obs.copy()
        if (t + 1) % 100 == 0:
            top = np.argsort(win)[::-1][:4]
            print(f"steps {t - 99}-{t}: max obs err {win.max():.2e} at components {top.tolist()} "
                  f"{[float('%.2e' % win[k]) for k in top]}", flush=True)
            win = np.zeros(0)


if __name__ == "__main__":
    main()

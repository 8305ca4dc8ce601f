"""Developer diagnostic: the free-running Gogoro env vs the oracle at ragged and
full batch sizes; at the first step whose obs differ by > 1e-3, print the env,
both observations and both root states."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, balance_policy, make_gpu_gogoro, parity_cfg  # noqa: E402


def run(n, seed, steps=80):
    env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
    orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
    obs_np = orc.a["obs_buf"].copy()
    prev_g = env.root_tensor.cpu().numpy().copy()
    prev_o = orc.a["root"].copy()
    for t in range(steps):
        act = balance_policy(obs_np)
        obs_d, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
        o_obs, o_rew, o_reset, _ = orc.step(act[:, 0])
        g_obs = obs_d["obs"].cpu().numpy()
        d = np.abs(g_obs - o_obs).max(axis=1)
        gr, orr = env.root_tensor.cpu().numpy(), orc.a["root"]
        if (d > 1e-3).any() or not np.isfinite(d).all():
            bad = np.nonzero(~(d <= 1e-3))[0]
            print(f"n={n} seed={seed} step {t}: bad envs {bad.tolist()} gpu finite {np.isfinite(g_obs).all()} "
                  f"oracle finite {np.isfinite(o_obs).all()}")
            for e in bad[:3]:
                print("  env", e, "gpu obs", g_obs[e], "oracle obs", o_obs[e])
                print("  gpu root", gr[e], "\n  orc root", orr[e])
                print("  prev gpu root", prev_g[e], "\n  prev orc root", prev_o[e])
                print("  resets gpu/orc", int(reset.cpu().numpy()[e]), int(o_reset[e]))
            return
        prev_g, prev_o = gr.copy(), orr.copy()
        obs_np = o_obs.copy()
    print(f"n={n} seed={seed}: {steps} steps within 1e-3")


if __name__ == "__main__":
    # argv: n:seed pairs run in order in this one process (default: the ragged test's order)
    pairs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(1, 51), (13, 63), (37, 87)]
    for n, seed in pairs:
        run(n, seed)

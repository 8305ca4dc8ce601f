"""Developer study (CPU): free-running Gogoro (balance policy, 64 envs, 1000
steps), the fp32 oracle build vs the fp64 oracle under each solver_type --
how far rounding alone carries the trajectories apart (max |obs| per
100-step window)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, balance_policy, parity_cfg  # noqa: E402


def run(solver, n=64, steps=1000, seed=0):
    def mk():
        c = parity_cfg(n)
        c["sim"]["physx"]["solver_type"] = solver
        return c
    a = OracleGogoro(mk(), NumpyDraws(seed))
    b = OracleGogoro(mk(), NumpyDraws(seed), precision="f32")
    win = []
    w = 0.0
    obs = a.a["obs_buf"].copy()
    for t in range(steps):
        act = balance_policy(obs)
        oa = a.step(act[:, 0])[0].copy()
        ob = b.step(act[:, 0])[0].copy()
        w = max(w, float(np.abs(oa - ob).max()))
        obs = oa
        if t % 100 == 99:
            win.append(w)
            w = 0.0
    print(f"solver_type {solver}: f32 vs f64 max |obs| per 100 steps:", " ".join(f"{x:.1e}" for x in win), flush=True)


if __name__ == "__main__":
    for s in (0, 1):
        run(s)

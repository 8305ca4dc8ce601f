"""Developer study (CPU, fp64 oracle only): where does the Gogoro spawn
landing amplify a 1e-6 state perturbation?  Runs the fp64 oracle env and a
copy whose initial root position / joint positions are shifted by 1e-6, under
the balance policy, and prints per step the max |obs| difference, the obs
component and env it sits in, and that env's root height / roll.

    python scripts/dev/tgs_landing_study.py [--solver 1] [--steps 80] [--envs 64]
"""
import argparse
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, balance_policy, parity_cfg  # noqa: E402


def mk(n, solver, seed, prec="f64", **over):
    c = parity_cfg(n, max_steps=1000)
    c["sim"]["physx"]["solver_type"] = solver
    for k, v in over.items():
        c["sim"]["physx"][k] = v
    return OracleGogoro(c, NumpyDraws(seed), precision=prec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solver", type=int, default=1)
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--seed", type=int, default=21)
    ap.add_argument("--every", type=int, default=1)
    ap.add_argument("--f32", action="store_true", help="compare the fp32 build instead of a perturbed fp64 run")
    a = ap.parse_args()
    n = a.envs
    ref = mk(n, a.solver, a.seed)
    if a.f32:
        p = mk(n, a.solver, a.seed, "f32")
    else:
        p = mk(n, a.solver, a.seed)
        rs2 = np.random.default_rng(a.seed + 999)
        p.a["root"][:, 0:3] += (1e-6 * rs2.choice([-1.0, 1.0], (n, 3))).astype(np.float32)
        p.a["dof_state"][:, 0] += (1e-6 * rs2.choice([-1.0, 1.0], p.a["dof_state"].shape[0])).astype(np.float32)
    obs = ref.a["obs_buf"].copy()
    worst = 0
    for t in range(a.steps):
        act = balance_policy(obs)
        ro = ref.step(act[:, 0])[0].copy()
        po = p.step(act[:, 0])[0].copy()
        d = np.abs(ro - po)
        e, c = np.unravel_index(np.argmax(d), d.shape)
        rd = np.abs(ref.a["root"] - p.a["root"]).max(axis=1)
        if t % a.every == 0 or d.max() > 1e-3:
            r = ref.a["root"][e]
            print(f"t {t:4d} obs {d.max():.2e} (env {e:2d} comp {c}) root {rd.max():.2e} (env {int(np.argmax(rd))}) "
                  f"z {r[2]:.4f} vz {r[9]:+.3f} prog {int(ref.a['progress_buf'][e])} obs0 {ro[e, 0]:+.4f}",
                  flush=True)
        worst = max(worst, d.max())
        obs = ro
    print("max", worst)


if __name__ == "__main__":
    main()

"""Developer study (CPU): one-step sensitivity of the walk env to float
rounding under each solver_type -- the fp32 build of the oracle physics
teacher-forced along the fp64 oracle's trajectory, max |obs| difference per
step window.  A GPU-vs-oracle one-step error of the same size is rounding,
not a kernel/oracle mismatch."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, walk_cfg  # noqa: E402


def run(solver, n=64, steps=120, seed=0, task="ThormangWalk"):
    def mk():
        c = walk_cfg(n, task)
        c["sim"].setdefault("physx", {})["solver_type"] = solver
        return c
    ref = OracleWalk(mk(), NumpyDraws(seed))
    f32 = OracleWalk(mk(), NumpyDraws(seed), precision="f32")
    rs = np.random.default_rng(seed + 100)
    worst = 0.0
    for t in range(steps):
        for k in ref.a:
            f32.a[k][...] = ref.a[k]
        act = rs.uniform(-0.5, 0.5, (n, ref.D)).astype(np.float32)
        o64 = ref.step(act)[0].copy()
        o32 = f32.step(act)[0].copy()
        worst = max(worst, float(np.abs(o64 - o32).max()))
    print(f"{task} solver_type {solver}: max one-step |obs f32 - obs f64| over {steps} steps, {n} envs: {worst:.3g}")


if __name__ == "__main__":
    for s in (0, 1):
        run(s)

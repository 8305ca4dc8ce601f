"""Developer study (GPU): teacher-forced walk steps, GPU and the fp32 oracle
build both compared with the fp64 oracle on identical inputs, under each
solver_type.  If the GPU's one-step error is of the fp32 build's size, the
GPU/oracle difference is rounding sensitivity, not a mismatch."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_oracle_from_gpu, walk_cfg  # noqa: E402


def run(solver, n, steps, seed=0, task="ThormangWalk"):
    def mk():
        c = walk_cfg(n, task)
        c["sim"].setdefault("physx", {})["solver_type"] = solver
        return c
    env = make_gpu_walk(mk(), NumpyDraws(seed))
    o64 = OracleWalk(mk(), NumpyDraws(seed), threads=16)
    o32 = OracleWalk(mk(), NumpyDraws(seed), threads=16, precision="f32")
    rs = np.random.default_rng(seed + 100)
    eg = e32 = 0.0
    ratio = []
    for t in range(steps):
        sync_oracle_from_gpu(o64, env)
        sync_oracle_from_gpu(o32, env)
        act = rs.uniform(-0.5, 0.5, (n, o64.D)).astype(np.float32)
        og = env.step(torch.from_numpy(act).to("cuda:0"))[0]["obs"].cpu().numpy()
        a = o64.step(act)[0].copy()
        b = o32.step(act)[0].copy()
        dg, d32 = np.abs(og - a).max(axis=1), np.abs(b - a).max(axis=1)
        eg, e32 = max(eg, float(dg.max())), max(e32, float(d32.max()))
        ratio.append(float(np.percentile(dg, 99.9)) / max(float(np.percentile(d32, 99.9)), 1e-12))
    print(f"{task} {n} envs solver_type {solver}: one-step max |gpu-f64| {eg:.3g}  max |f32-f64| {e32:.3g}  "
          f"p99.9 ratio gpu/f32 median {np.median(ratio):.2f}", flush=True)


if __name__ == "__main__":
    for s in (0, 1):
        run(s, 8192, 60)

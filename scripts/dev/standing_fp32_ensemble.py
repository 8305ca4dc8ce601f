"""Developer probe (CPU only): when does an fp32 computation of the standing
walk (tests/test_gpu_parity_long.py's workload: 32 envs, zero actions, 1000
free-running steps, seed 21) leave the 1e-3 band of the fp64 reference?  The
fp32 oracle build unperturbed (the test's rounding control) and K fp32 builds
whose initial joint positions and pelvis height are moved by +-eps (eps
1e-7: below an fp32 ulp of those values, i.e. the same computation rounded
differently): the spread of their departure steps is how far apart two
equally accurate fp32 evaluations of this chaotic trajectory part ways.

    python scripts/dev/standing_fp32_ensemble.py [K] [eps] [steps]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, perturbed_walk_oracle, walk_cfg  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-7
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
n, seed = 32, 21
ref = OracleWalk(walk_cfg(n), NumpyDraws(seed))
runs = {"fp32 (the control)": OracleWalk(walk_cfg(n), NumpyDraws(seed), precision="f32")}
for k in range(K):
    runs[f"fp32 +-{eps:g} #{k}"] = perturbed_walk_oracle(walk_cfg(n), seed, 100 + k, eps, precision="f32")
dep = {k: None for k in runs}
act = np.zeros((n, ref.D), np.float32)
for t in range(steps):
    r_obs, r_rew, r_reset, _ = ref.step(act)
    r_obs, r_rew, r_reset = r_obs.copy(), r_rew.copy(), r_reset.copy()
    for k, o in runs.items():
        obs, rew, reset, _ = o.step(act)
        if dep[k] is None and (np.abs(obs - r_obs).max() > 1e-3 or np.abs(rew - r_rew).max() > 1e-3 or
                               not np.array_equal(reset, r_reset)):
            dep[k] = t
print(f"standing walk, {n} envs x {steps} steps, seed {seed}: first step each fp32 run leaves 1e-3 of fp64 "
      "(obs or reward) or changes a reset flag")
for k, v in dep.items():
    print(f"  {k:22s} {v}")
d = np.array([v if v is not None else steps for v in dep.values()], float)
print(f"  spread: min {d.min():.0f}  median {np.median(d):.0f}  max {d.max():.0f}")

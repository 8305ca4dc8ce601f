"""Developer probe (CPU only): how often does a rounding-level perturbation of
the fp64 oracle itself change a reset flag of the standing walk
(tests/test_gpu_parity_long.py's standing workload, 1000 free-running steps)?
K runs of the fp64 oracle, each with its own random 1e-7 perturbation of the
joint positions and the pelvis height, and the fp32 build, against the
unperturbed fp64 run: per run the first step over 1e-3 and the first reset
mismatch with the envs' termination margins there.

    python scripts/dev/standing_chaos_cpu.py [K] [num_envs] [steps] [seed] [eps]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleWalk, perturbed_walk_oracle, walk_cfg  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 21
eps = float(sys.argv[5]) if len(sys.argv) > 5 else 1e-7
ref = OracleWalk(walk_cfg(n), NumpyDraws(seed))
runs = {}
for k in range(K):
    runs[f"fp64+{eps:g}#{k}"] = perturbed_walk_oracle(walk_cfg(n), seed, k, eps)
runs["fp32"] = OracleWalk(walk_cfg(n), NumpyDraws(seed), precision="f32")
res = {k: {"horizon": None, "reset_diff": None} for k in runs}
act = np.zeros((n, ref.D), np.float32)
for t in range(steps):
    r_obs, _, r_reset, _ = ref.step(act)
    r_obs, r_reset = r_obs.copy(), r_reset.copy()
    for k, o in runs.items():
        obs, _, reset, _ = o.step(act)
        if res[k]["horizon"] is None and np.abs(obs - r_obs).max() > 1e-3:
            res[k]["horizon"] = t
        if res[k]["reset_diff"] is None and not np.array_equal(reset, r_reset):
            bad = np.nonzero(reset != r_reset)[0]
            margin = np.minimum(np.abs(r_obs[bad, 0] - ref.p.termination_height),
                                np.abs(-r_obs[bad, 9] - ref.p.termination_up))
            res[k]["reset_diff"] = (t, bad.tolist(), [round(float(m), 6) for m in margin])
print(f"standing walk, {n} envs x {steps} steps, seed {seed}; resets in the reference run: "
      f"{int(ref.a['reset_buf'].sum())} pending at the end")
for k, r in res.items():
    print(f"{k:16s} first step > 1e-3: {r['horizon']}   first reset mismatch (step, envs, margins): {r['reset_diff']}")

"""Developer study (GPU): the 1000-step free-running ensemble rule of
tests/test_gpu_parity_long.py on more seeds -- for each workload and seed,
the GPU's departure step from the fp64 reference (obs or reward over 1e-3,
or a reset flag changed) against the 9 fp32 evaluations' (the control and 8
builds started 1e-7 away), and the GPU's rank among them.

    python scripts/dev/r5_long_seeds.py [seeds...]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import gogoro_env_vs_oracle, walk_env_vs_oracle  # noqa: E402

import os
seeds = [int(x) for x in sys.argv[1:]] or [1, 2, 3]
WORK = os.environ.get("WORK", "walk,walkdr,gogoro").split(",")


def summary(name, seed, err):
    n = err["steps"]
    deps = sorted([err.get("ctl_first_bad", n)] + [d if d is not None else n for d in err["f32_departures"]])
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    rank = int(np.searchsorted(deps, gpu, side="right"))
    ok = gpu >= deps[2]
    print(f"{name:22s} seed {seed:3d}: gpu departs {gpu:5d}  fp32 {deps}  rank {rank}/9  "
          f"obs {err['obs']:.2e} rew {err['rew']:.2e} resets {err['resets']}  {'ok' if ok else 'EARLY'}", flush=True)


for seed in seeds:
  if "walk" in WORK:
    summary("walk U(0.3)", seed, walk_env_vs_oracle(num_envs=64, steps=1000, seed=100 + seed, amp=0.3, control=True,
                                                    f32_ensemble=8))
  if "walkdr" in WORK:
    summary("walkDR pushes", seed, walk_env_vs_oracle(num_envs=32, steps=1000, seed=200 + seed, task="ThormangWalkDR",
                                                      control=True, f32_ensemble=8))
  if "gogoro" in WORK:
    rs = np.random.default_rng(300 + seed)
    summary("gogoro U(1)", seed, gogoro_env_vs_oracle(num_envs=64, steps=1000, seed=300 + seed, control=True,
                                                      f32_ensemble=8,
                                                      policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32)))

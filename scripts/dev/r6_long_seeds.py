"""Developer study (GPU), VERDICT r5 items 1-2: the 1000-step free-running
ensemble comparisons on many seeds -- per workload and seed, the GPU's
departure step from the fp64 reference (obs or reward over 1e-3, or a reset
flag changed) against the 9 fp32 evaluations' (the fp32 control and 8 fp32
builds started 1e-7 away), the GPU's rank among them, and whether it meets
round 6's bars: the median fp32 evaluation (humanoid), the fp32 control
(scooter, whose ensemble is degenerate).

    WORK=walk,walkdr,stand,gogoro python scripts/dev/r6_long_seeds.py [seeds...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import gogoro_env_vs_oracle, walk_env_vs_oracle  # noqa: E402

seeds = [int(x) for x in sys.argv[1:]] or [1, 2, 3, 4, 5, 6]
WORK = os.environ.get("WORK", "walk,walkdr,stand,gogoro").split(",")


def summary(name, seed, err, bar):
    n = err["steps"]
    ctl = err.get("ctl_first_bad", n)
    deps = sorted([ctl] + [d if d is not None else n for d in err["f32_departures"]])
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    rank = int(np.searchsorted(deps, gpu, side="right"))
    need = deps[4] if bar == "median" else ctl
    print(f"{name:16s} seed {seed:3d}: gpu {gpu:5d}  fp32 {deps}  ctl {ctl:5d}  rank {rank}/9  "
          f"{'ok' if gpu >= need else 'EARLY'} (bar: {bar} {need})", flush=True)


for seed in seeds:
    if "walk" in WORK:
        summary("walk U(0.3)", seed, walk_env_vs_oracle(num_envs=64, steps=1000, seed=100 + seed, amp=0.3,
                                                        control=True, f32_ensemble=8), "median")
    if "walkdr" in WORK:
        summary("walkDR pushes", seed, walk_env_vs_oracle(num_envs=32, steps=1000, seed=200 + seed,
                                                          task="ThormangWalkDR", control=True, f32_ensemble=8), "median")
    if "stand" in WORK:
        summary("walk standing", seed, walk_env_vs_oracle(num_envs=32, steps=1000, seed=400 + seed, amp=0.0,
                                                          control=True, f32_ensemble=8), "median")
    if "gogoro" in WORK:
        rs = np.random.default_rng(300 + seed)
        summary("gogoro U(1)", seed, gogoro_env_vs_oracle(
            num_envs=64, steps=1000, seed=300 + seed, control=True, f32_ensemble=8,
            policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32)), "control")

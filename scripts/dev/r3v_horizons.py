"""Probe: free-running walk (DR) horizons vs the fp64 oracle env."""
import sys, json
sys.path.insert(0, ".")
from tests.gpu_harness import walk_env_vs_oracle
for task, seed, steps in [("ThormangWalkDR", 6, 150), ("ThormangWalkDR", 7, 200), ("ThormangWalk", 9, 300)]:
    e = walk_env_vs_oracle(num_envs=32, steps=steps, seed=seed, task=task)
    print(task, seed, steps, json.dumps({k: (float(v) if not isinstance(v, bool) else v) for k, v in e.items()}), flush=True)

"""Round-4 developer run (GPU): the 600-step free-running walk parity run
(64 envs, seed 21, random actions U(+-0.3), the fp32 control beside the fp64
oracle) under each solver_type; prints the error dict per solver."""
import sys

sys.path.insert(0, ".")
from tests.gpu_harness import walk_env_vs_oracle, within  # noqa: E402

for st in map(int, (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")):
    err = walk_env_vs_oracle(num_envs=64, steps=600, seed=21, amp=0.3, control=True, solver_type=st)
    print(f"solver_type {st}: within obs {within(err)} rew {within(err, 'rew')}", {k: v for k, v in err.items()}, flush=True)

"""Round-4 developer run (GPU): the 8192-env teacher-forced walk (100 steps,
seed 11, test_gpu_walk_8192_envs_step_matches_oracle) with the fp32 oracle
control beside the fp64 one, under each solver_type given (argv[1], default
"1"); TG_LIB_PATH selects a developer build of libtgsim."""
import os
import sys

sys.path.insert(0, ".")
from tests.gpu_harness import walk_forced  # noqa: E402

lib = os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so"))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
for st in map(int, (sys.argv[1] if len(sys.argv) > 1 else "1").split(",")):
    err = walk_forced(num_envs=n, steps=100, seed=11, control=True, solver_type=st)
    print(f"{lib} solver_type {st} n {n}:", {k: (round(v, 7) if isinstance(v, float) else v) for k, v in err.items()},
          flush=True)

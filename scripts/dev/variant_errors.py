"""Developer probe (GPU): the parity runs that sit nearest the 1e-3 bar,
under the library TG_LIB_PATH names (default libtgsim.so), one line each:

  paper_forced   GogoroPaper, flags flipped, 300 teacher-forced steps
                 (test_gpu_paper_free_base_step_matches_oracle_along_300_steps)
  walk_forced    ThormangWalk 8192 envs, 100 teacher-forced steps, fp32 control
  walk_dr        ThormangWalkDR 32 envs, 200 free-running steps
  walk_stand     ThormangWalk standing 32 envs, 1000 free-running steps, fp32 control

    TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_x.so python scripts/dev/variant_errors.py paper_forced,walk_forced [solver]
"""
import os
import sys

sys.path.insert(0, ".")

lib = os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so"))
which = (sys.argv[1] if len(sys.argv) > 1 else "paper_forced,walk_forced,walk_dr,walk_stand").split(",")
st = int(sys.argv[2]) if len(sys.argv) > 2 else None


def short(err):
    keys = ("obs", "rew", "obs_f32", "rew_f32", "reset_equal", "first_bad_step", "resets")
    return {k: (float("%.3g" % err[k]) if isinstance(err[k], float) else err[k]) for k in keys if k in err}


for w in which:
    if w == "paper_forced":
        from tests.test_gpu_paper import FLIPPED, _env_vs_oracle
        err = _env_vs_oracle(FLIPPED, steps=300, forced=True)
    elif w == "walk_forced":
        from tests.gpu_harness import walk_forced
        err = walk_forced(num_envs=8192, steps=100, seed=11, control=True, solver_type=st)
    elif w == "walk_dr":
        from tests.gpu_harness import walk_env_vs_oracle
        err = walk_env_vs_oracle(num_envs=32, steps=200, seed=7, task="ThormangWalkDR", control=True, solver_type=st)
    elif w == "walk_stand":
        from tests.gpu_harness import walk_env_vs_oracle
        err = walk_env_vs_oracle(num_envs=32, steps=1000, seed=21, amp=0.0, control=True, solver_type=st)
    print(f"{lib} {w} solver={st}: {short(err)}", flush=True)

"""north_star's parity criterion -- obs / reward / done within 1e-3 over 1000
steps -- FREE-RUNNING (no re-sync of the oracle from the GPU state), on the
configurations whose dynamics do not amplify 1e-7-size rounding differences:

* Gogoro with a fixed base (the reference's DEBUGFIXBASE switch,
  tasks/gogoro_new.py:22,206): steering drive, wheels, free grip joints;
* ThormangWalk with a fixed base hung clear of the ground, random actions;
* ThormangWalk standing on the ground under its PD drives (zero actions):
  free base, both feet in contact for 1000 steps;
* Gogoro with a free base under the balance controller: falls, resets and
  re-spawns included, as long as no fall happens within rounding of the tilt
  threshold (then the reset draw streams of the two sides part, see
  scripts/parity_drift.py and DESIGN.md §2).

plus the reference's domain randomisation live on the Gogoro path (link
masses x U[0.95,1.05], gravity x U[0.95,1.05] every 600 frames; the oracle
simulates the models the GPU env drew, tests/gpu_harness.py sync_dr).
scripts/parity_drift.py measures, for the chaotic configurations, how far a
1e-6 perturbation of the fp64 oracle and an fp32 build of the oracle drift
from it (profiles/r2/drift_*.txt)."""
import pytest
import torch
from tests.gpu_harness import brief, within

pytestmark = pytest.mark.gpu


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def test_gpu_gogoro_fixed_base_free_running_1000_steps():
    _cuda()
    from tests.gpu_harness import balance_policy, gogoro_env_vs_oracle
    err = gogoro_env_vs_oracle(num_envs=64, steps=1000, seed=31, policy=balance_policy, fix_base=True)
    print(brief(err))
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    assert err["resets"] >= 64          # every env times out at step 999 and re-spawns
    # joint state: the wheels spin freely on the fixed base and their angles
    # grow without bound, so the joint error is relative to |q| (the fp32 ulp
    # of a large angle accumulates over 3000 substeps)
    assert err["dof_rel"] < 1e-3, err


def test_gpu_walk_fixed_base_free_running_1000_steps():
    _cuda()
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=32, steps=1000, seed=32, fix_base=True, spawn_height=1.3, amp=0.3)
    print(brief(err))
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    assert err["root"] < 1e-3 and err["dof"] < 1e-3, err


def test_gpu_walk_random_actions_free_running_1000_steps():
    """The headline walk free-running for north_star's 1000 steps with falls
    and re-spawns (64 envs, random actions U(-0.3, 0.3), seed 21; VERDICT r4:
    no walk test ran 1000 free-running steps with falls).  Falling humanoids
    amplify rounding: the fp32 oracle build's own reset flags desync from the
    fp64 reference at step 319, so no fp32 computation -- the GPU's included
    -- tracks fp64 to 1e-3 for all 1000 steps.  As for the standing walk, the
    yardstick is what fp32 rounding alone does: the control and 8 fp32 builds
    started 1e-7 away (below an fp32 ulp) give 9 departure steps, and the GPU
    must not depart before the third-earliest (obs and reward within 1e-3,
    identical reset flags, at every step before it).  The steps after it are
    reported, not asserted (round 4's drift study: the GPU leaves 1e-3 at
    step 723, the fp32 build at 320; profiles/r4/drift_walk_root_relative.txt).
    A single-seed regression guard: on other seeds the GPU's departure ranks
    anywhere among the fp32 evaluations' (profiles/r5/long_seeds.txt)."""
    _cuda()
    import numpy as np
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=64, steps=1000, seed=21, amp=0.3, control=True, f32_ensemble=8)
    n = err["steps"]
    deps = sorted([err.get("ctl_first_bad", n)] + [d if d is not None else n for d in err["f32_departures"]])
    hz = deps[2]
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    err.update(f32_sorted=deps, horizon=hz, gpu_departure=gpu,
               gpu_rank=int(np.searchsorted(deps, gpu, side="right")),
               obs_pre_horizon=float(np.max(err["_obs_t"][:hz])), rew_pre_horizon=float(np.max(err["_rew_t"][:hz])))
    print(brief(err))
    assert err["resets"] > 0, brief(err)
    assert hz >= 100, brief(err)
    assert gpu >= hz, brief(err)
    assert err["obs_pre_horizon"] < 1e-3 and err["rew_pre_horizon"] < 1e-3, brief(err)


def test_gpu_walk_dr_pushes_free_running_1000_steps():
    """ThormangWalkDR (random pushes on top of the falls), 32 envs, 1000
    free-running steps, under the same fp32-ensemble rule as the plain walk
    (test_gpu_walk_random_actions_free_running_1000_steps): the GPU must not
    depart from the fp64 reference (obs or reward over 1e-3, or a reset flag
    changed) before the third-earliest of 9 fp32 evaluations of the same
    episode (the control and 8 fp32 builds started 1e-7 away).  A single-seed
    regression guard (other seeds: profiles/r5/long_seeds.txt)."""
    _cuda()
    import numpy as np
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=32, steps=1000, seed=7, task="ThormangWalkDR", control=True, f32_ensemble=8)
    n = err["steps"]
    deps = sorted([err.get("ctl_first_bad", n)] + [d if d is not None else n for d in err["f32_departures"]])
    hz = deps[2]
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    err.update(f32_sorted=deps, horizon=hz, gpu_departure=gpu,
               gpu_rank=int(np.searchsorted(deps, gpu, side="right")),
               obs_pre_horizon=float(np.max(err["_obs_t"][:hz])), rew_pre_horizon=float(np.max(err["_rew_t"][:hz])))
    print(brief(err))
    assert err["resets"] > 0, brief(err)
    assert hz >= 50, brief(err)
    assert gpu >= hz, brief(err)
    assert err["obs_pre_horizon"] < 1e-3 and err["rew_pre_horizon"] < 1e-3, brief(err)


def test_gpu_walk_standing_free_running_1000_steps():
    """ThormangWalk standing (zero actions: the PD-held default pose), 32 envs,
    1000 free-running steps; some spawn poses topple (20 falls with seed 21).

    A toppling humanoid amplifies rounding: the fp64 reference itself, started
    from states perturbed by 1e-7, leaves the 1e-3 band between steps 580 and
    853 (profiles/r4/standing_chaos_cpu.txt).  VERDICT r4 asked that the GPU
    not leave 1e-3 before the fp32 control does -- one sample against one
    sample.  Round 5 measures what fp32 rounding alone does here: beside the
    fp32 control run 8 fp32 builds whose initial state is moved by 1e-7
    (below an fp32 ulp of it: the same computation rounded differently,
    scripts/dev/standing_fp32_ensemble.py, profiles/r5/standing_fp32_ensemble.txt);
    their departure steps (obs or reward over 1e-3 of fp64, or a reset flag
    changed) are 572, 579, 589 and 637 for the other six and the control.
    The bar: the GPU must not depart before the third-earliest of those 9
    equally accurate fp32 evaluations (the ensemble's lower quartile), i.e.
    obs and reward within 1e-3 and identical reset flags at every step
    before it; time-out flags agree throughout.  Every yardstick's departure
    is reported (``f32_departures``, ``ctl_first_bad``, ``pert_departures``)."""
    _cuda()
    import numpy as np
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=32, steps=1000, seed=21, amp=0.0, control=True, perturbed=3, f32_ensemble=8)
    n = err["steps"]
    deps = sorted([err.get("ctl_first_bad", n)] + [d if d is not None else n for d in err["f32_departures"]])
    hz = deps[2]   # the third-earliest of the 9 fp32 departures
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    err.update(f32_sorted=deps, horizon=hz, gpu_departure=gpu,
               gpu_rank=int(np.searchsorted(deps, gpu, side="right")),
               obs_pre_horizon=float(np.max(err["_obs_t"][:hz])), rew_pre_horizon=float(np.max(err["_rew_t"][:hz])))
    print(brief(err))
    assert err["resets"] < 32, brief(err)
    assert hz >= 100, brief(err)                      # the yardstick itself is sane
    assert gpu >= hz, brief(err)
    assert err["obs_pre_horizon"] < 1e-3 and err["rew_pre_horizon"] < 1e-3, brief(err)
    assert err["timeout_equal"], brief(err)


def test_gpu_gogoro_free_base_free_running_1000_steps():
    _cuda()
    from tests.gpu_harness import balance_policy, gogoro_env_vs_oracle
    err = gogoro_env_vs_oracle(num_envs=32, steps=1000, seed=21, policy=balance_policy)
    print(brief(err))
    assert err["resets"] > 32           # falls and re-spawns happen along the way
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_domain_randomisation_matches_oracle():
    """The reference's randomization_params live on both sides: 150 free-running
    steps, then 1000 teacher-forced steps (which cross the 600-frame gravity
    resample)."""
    _cuda()
    from tests.gpu_harness import balance_policy, gogoro_env_vs_oracle, gogoro_forced
    err = gogoro_env_vs_oracle(num_envs=64, steps=150, seed=41, policy=balance_policy, dr=True)
    print(brief(err))
    lo, hi = err["mass_scale_range"]
    assert 0.95 <= lo < 0.96 and 1.04 < hi <= 1.05, err      # masses really randomised
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    err = gogoro_forced(num_envs=64, steps=1000, seed=42, dr=True)
    print(brief(err))
    assert err["gravity"] != [0.0, 0.0, -9.81], err            # resampled at frame 600
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_free_base_random_actions_free_running():
    """The bench's own action distribution (U(-1,1) steering increments every
    step) on the free base, free running, 100 steps at the strict bar over
    every step (every env falls and re-spawns at least once).  Round 3 cut
    this run at 100 steps because the GPU then left 1e-3 at step 121; since
    round 4's TGS conditioning fixes the same workload holds 1e-3 for 1000
    steps (test_gpu_gogoro_random_actions_free_running_1000_steps)."""
    _cuda()
    import numpy as np
    from tests.gpu_harness import gogoro_env_vs_oracle
    rs = np.random.default_rng(77)
    err = gogoro_env_vs_oracle(num_envs=64, steps=100, seed=22,
                               policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32))
    print(brief(err))
    assert err["resets"] >= 64
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_random_actions_free_running_1000_steps():
    """The bench's own action distribution on the free base, free running for
    north_star's 1000 steps (64 envs, seed 22; every env falls and re-spawns
    about 23 times), held to 1e-3 on every step with identical reset flags,
    as is the fp32 control beside it on this seed.  This is one seed's
    regression guard, not a general claim: on 6 other seeds
    (scripts/dev/r5_long_seeds.py, profiles/r5/long_seeds.txt) fp32
    computations leave the 1e-3 band at discrete events (a fall decided by a
    threshold tie, a drive crossing its effort limit) -- the
    fp32 oracle build on 4 of them, the GPU on all 6, first on 5."""
    _cuda()
    import numpy as np
    from tests.gpu_harness import gogoro_env_vs_oracle
    rs = np.random.default_rng(77)
    err = gogoro_env_vs_oracle(num_envs=64, steps=1000, seed=22, control=True,
                               policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32))
    print(brief(err))
    assert err["resets"] >= 64, brief(err)
    assert within(err) and within(err, "rew"), brief(err)
    assert err["reset_equal"] and err["timeout_equal"], brief(err)

def test_gpu_walk_random_actions_free_running_600_steps():
    """The headline walk free-running with falls and re-spawns: 64 envs,
    random actions U(-0.3, 0.3), 600 steps -- the drift study's workload
    (`scripts/parity_drift.py walk`, profiles/r3/drift_walk.txt: the GPU and
    the fp32 oracle build both leave the 1e-3 band near step 700, chaos after
    the falls), at the north_star bar up to there.  The fp32 oracle build runs
    beside it as the rounding control: a numerically harmless kernel change
    moves this chaotic trajectory (storing two rotation columns and forming the
    third by a cross product left 1e-3 at step 211), so the bar is 1e-3 up to the
    control's first departure from the fp64 reference (its reset flags desync
    at step 319): the GPU is held to 1e-3 at every step before it
    (tests/gpu_harness.within) and reported after it (round 4: the GPU stayed
    within 6.4e-4 obs / 4.0e-4 reward over all 600 steps)."""
    _cuda()
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=64, steps=600, seed=21, amp=0.3, control=True)
    print(brief(err))
    assert err["resets"] > 0, err            # envs fall and re-spawn along the way
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err

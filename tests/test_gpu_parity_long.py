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
from it (profiles/r2/drift_*.txt).  The chaotic 1000-step runs (walk with
falls, walk with DR pushes, standing walk, scooter under random steering)
are in tests/test_gpu_parity_seeds.py, on 7-10 seeds each against the fp32
rounding ensemble (round 6: they replaced the single-seed guards here)."""
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
    steps on 10 seeds (tests/test_gpu_parity_seeds.py)."""
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

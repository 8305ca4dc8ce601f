"""north_star's 1000-step free-running bar on many seeds.

Every run here is chaotic: falling humanoids, and a scooter under the bench's
random steering that falls and re-spawns ~23 times per env.  No fp32
computation tracks the fp64 oracle to 1e-3 for 1000 steps on every seed -- the
oracle's own fp32 build does not -- so the yardstick is what fp32 rounding
alone does on the same episode: the fp32 control and 8 fp32 builds started
1e-7 away (below an fp32 ulp of the state), 9 "fp32 evaluations" whose
departure steps (obs or reward over 1e-3 of fp64, or a reset flag changed)
the GPU's departure is ranked among (rank = how many of the 9 left at or
before the GPU; 9 = the GPU left last or never).

The bar is a statistical one, because a per-seed bar is a coin flip for ANY
fp32 computation: each of the 9 fp32 evaluations, judged against the median
of the others, fails about half the seeds.  A GPU whose rounding is as good
as the oracle's fp32 build is exchangeable with the 9 evaluations, its rank
uniform on 0..9 (mean 4.5, sd 2.87); a GPU with a systematic rounding excess
ranks low.  Asserted:

* humanoid (walk U(+-0.3), walk with DR pushes, standing walk; 7 seeds
  each): the GPU's mean rank over the seeds >= 2.7 per workload (the
  one-sided 5 % bound of a uniform rank, 4.5 - 1.645 x 2.87 / sqrt 7) and
  >= 3.47 over all 21 runs;
* scooter (10 seeds): its 9 fp32 evaluations are degenerate (the dynamics
  contract a 1e-7 perturbation; each departure is a discrete fp32-vs-fp64
  event), so the race is against the fp32 control: the GPU leaves first on
  no more seeds than the control leaves first.  Round 5's kernel lost this
  race 5 to 1 on seeds 1-6 (profiles/r5/long_seeds.txt); round 6's
  contact-local rows removed the excess that made it.

Every seed also holds the GPU within 1e-3 at every step before its own
departure and requires that departure after step 100 (a GPU that leaves in
the first 100 steps fails outright).  Every seed's departures are printed."""
import numpy as np
import pytest
import torch

from tests.gpu_harness import gogoro_env_vs_oracle, walk_env_vs_oracle

pytestmark = pytest.mark.gpu

WALK_SEEDS = [21, 101, 102, 103, 104, 105, 106]
DR_SEEDS = [7, 201, 202, 203, 204, 205, 206]
STAND_SEEDS = [21, 401, 402, 403, 404, 405, 406]
GOGORO_SEEDS = [301, 302, 303, 304, 305, 306, 307, 308, 309, 322]
_ranks = {}


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def departures(err):
    """(GPU departure, the control's, the 9 fp32 departures sorted, the GPU's rank)."""
    n = err["steps"]
    ctl = err.get("ctl_first_bad", n)
    deps = sorted([ctl] + [d if d is not None else n for d in err["f32_departures"]])
    gpu = min(err.get("first_bad_step", n), err.get("reset_diff_step", n) if not err["reset_equal"] else n)
    return gpu, ctl, deps, int(np.searchsorted(deps, gpu, side="right"))


def _check_seed(name, seed, err):
    gpu, ctl, deps, rank = departures(err)
    pre = err["_obs_t"][:gpu], err["_rew_t"][:gpu]
    print(f"{name:14s} seed {seed:4d}: gpu {gpu:5d}  control {ctl:5d}  fp32 {deps}  rank {rank}/9", flush=True)
    assert err["resets"] > 0
    assert gpu >= 100, (name, seed, gpu, deps)
    assert max(pre[0]) < 1e-3 and max(pre[1]) < 1e-3, (name, seed)
    return gpu, ctl, rank


def _humanoid(name, seeds, run):
    _cuda()
    ranks = [_check_seed(name, s, run(s))[2] for s in seeds]
    _ranks[name] = ranks
    mean = float(np.mean(ranks))
    print(f"{name}: ranks {ranks}, mean {mean:.2f} (bar 2.7; uniform 4.5)", flush=True)
    assert mean >= 2.7, ranks


def test_gpu_walk_random_actions_1000_steps_seeds():
    _humanoid("walk U(0.3)", WALK_SEEDS,
              lambda s: walk_env_vs_oracle(num_envs=64, steps=1000, seed=s, amp=0.3, control=True, f32_ensemble=8))


def test_gpu_walk_dr_pushes_1000_steps_seeds():
    _humanoid("walkDR pushes", DR_SEEDS,
              lambda s: walk_env_vs_oracle(num_envs=32, steps=1000, seed=s, task="ThormangWalkDR", control=True,
                                           f32_ensemble=8))


def test_gpu_walk_standing_1000_steps_seeds():
    _humanoid("walk standing", STAND_SEEDS,
              lambda s: walk_env_vs_oracle(num_envs=32, steps=1000, seed=s, amp=0.0, control=True, f32_ensemble=8))


def test_gpu_humanoid_ranks_pooled():
    """The three humanoid workloads' 21 runs together: mean rank >= 3.47 (the
    one-sided 5 % bound of 21 uniform ranks).  Needs the three tests above
    (same session); skipped when run alone."""
    if len(_ranks) < 3:
        pytest.skip("run with the three humanoid seed tests")
    allr = [r for v in _ranks.values() for r in v]
    print(f"humanoid pooled: {len(allr)} runs, mean rank {np.mean(allr):.2f}", flush=True)
    assert np.mean(allr) >= 3.47, _ranks


def test_gpu_gogoro_random_actions_1000_steps_seeds():
    """The bench's action distribution (U(-1,1) steering every step) on the
    free base, 64 envs, 1000 steps, 10 seeds: the GPU may not lose the
    departure race against the fp32 control (leave 1e-3 first on more seeds
    than the control leaves first)."""
    _cuda()
    gpu_first = ctl_first = 0
    for s in GOGORO_SEEDS:
        rs = np.random.default_rng(s)
        err = gogoro_env_vs_oracle(num_envs=64, steps=1000, seed=s, control=True, f32_ensemble=8,
                                   policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32))
        assert err["resets"] >= 64 * 10
        gpu, ctl, _ = _check_seed("gogoro U(1)", s, err)
        gpu_first += gpu < ctl
        ctl_first += ctl < gpu
    print(f"gogoro: the GPU leaves first on {gpu_first} seeds, the fp32 control on {ctl_first}", flush=True)
    assert gpu_first <= ctl_first, (gpu_first, ctl_first)

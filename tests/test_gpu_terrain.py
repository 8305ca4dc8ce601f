"""Terrain contact on the GPU: the HIP step kernel's
heightfield path against the fp64 oracle on a Perlin terrain, and the incline
known answers (static when mu > tan(theta), sliding at g(sin - mu cos) when
not) through the C-ABI."""
import numpy as np
import pytest
import torch

from tests import physics_models as pm
from tests.oracle_lib import physics_step, set_heightfield
from tests.gpu_harness import within
from tests.gpu_harness import maxerr

pytestmark = pytest.mark.gpu


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def _gpu_sim(model, sp, n, root, dof, props, pt, vt):
    from tests.test_gpu_physics import gpu_sim
    return gpu_sim(model, sp, n, root, dof, props, pt, vt)


def _perlin(seed, shape=(64, 64)):
    from thormang_isaacgym_amd.tasks.terrain import Terrain
    return Terrain(torch.Generator().manual_seed(seed), shape=shape).heightsamples.numpy()


@pytest.mark.parametrize("shape", ["sphere", "box"])
def test_gpu_terrain_contact_matches_oracle(shape):
    """32 bodies dropped on a Perlin terrain, 200 steps, teacher-forced: before
    every step the oracle takes the GPU state, so each step's contact
    resolution is compared from identical inputs.  (Free-running trajectories
    of bodies rolling over the piecewise-planar mesh separate by design: a
    body crossing a triangle edge a step earlier on one side sees a jump in
    the contact normal -- scripts/terrain_diag.py shows both.)  Tolerances:
    positions/orientations 1e-4, velocities 5e-3 (16 PGS sweeps on four
    redundant box corners are not converged; fp32 vs fp64 W moves the
    residual)."""
    _cuda()
    n, steps = 32, 200
    m = pm.sphere_body(0.1) if shape == "sphere" else pm.box_body()
    desc, sp, root, dof, props, pt, vt = pm.sim(m, n=n, dt=0.01, substeps=2, ground_friction=0.8)
    hf = _perlin(7)
    hs, org = 0.5, (-4.0, -6.0)
    rs = np.random.default_rng(1)
    xy = rs.uniform(2.0, 24.0, (n, 2))
    from thormang_isaacgym_amd.tasks.terrain import surface_height
    tz = surface_height(hf, hs, 1.0, xy[:, 0] - org[0], xy[:, 1] - org[1])
    root[:, 0:2] = xy
    root[:, 2] = np.maximum(tz, 0.0) + rs.uniform(0.15, 0.4, n)
    root[:, 7:9] = rs.normal(0, 0.5, (n, 2))
    g = _gpu_sim(m, sp, n, root, dof, props, pt, vt)
    g.set_heightfield(hf, hs, 1.0, org[0], org[1], friction=0.9)
    set_heightfield(hf, hs, 1.0, org[0], org[1], friction=0.9)
    pose_err = vel_err = 0.0
    try:
        for _ in range(steps):
            r = g.root_state.cpu().numpy().copy()
            d = g.dof_state.cpu().numpy().copy()
            physics_step(desc, sp, r, d, props, pt, vt)
            g.simulate()
            gr = g.root_state.cpu().numpy()
            pose_err = max(pose_err, maxerr(gr[:, :7], r[:, :7]))
            vel_err = max(vel_err, maxerr(gr[:, 7:], r[:, 7:]))
    finally:
        set_heightfield(None)
    print(shape, "pose", pose_err, "vel", vel_err)
    assert np.isfinite(gr).all()
    # on (not through) the terrain: every body's lowest point is within 1 cm of the surface
    tz_end = np.maximum(surface_height(hf, hs, 1.0, gr[:, 0] - org[0], gr[:, 1] - org[1]), 0.0)
    assert (gr[:, 2] - tz_end > 0.02).all()
    assert pose_err < 1e-4 and vel_err < 5e-3, (pose_err, vel_err)


def _incline_run(theta, mu, steps):
    """4 boxes resting on z = tan(theta) x; shape, terrain and plane friction mu
    (the compiled kat_box has mu = 1: friction is set per env at run time)."""
    h = np.repeat((np.tan(theta) * np.arange(80) * 0.5)[:, None], 80, 1).astype(np.float32)
    desc, sp, root, dof, props, pt, vt = pm.sim(pm.box_body(), n=4, dt=0.005, substeps=1, ground_friction=mu)
    nrm = np.array([-np.sin(theta), 0.0, np.cos(theta)])
    for e in range(4):
        root[e, :3] = np.array([20.0, 5.0 + 5 * e, np.tan(theta) * 20.0]) + 0.05 * nrm
        root[e, 3:7] = [0.0, np.sin(-theta / 2), 0.0, np.cos(-theta / 2)]
    g = _gpu_sim(pm.box_body(), sp, 4, root, dof, props, pt, vt)
    g.set_shape_friction_indexed(torch.full((4, 1), float(mu), device="cuda:0"), torch.arange(4))
    g.set_heightfield(h, 0.5, 1.0, 0.0, 0.0, friction=mu)
    traj = []
    for _ in range(steps):
        g.simulate()
        traj.append(g.root_state.cpu().numpy().copy())
    return np.array(traj), sp


def test_gpu_box_sticks_on_incline():
    _cuda()
    theta = 0.3
    traj, _ = _incline_run(theta, np.tan(theta) + 0.4, 120)
    assert np.linalg.norm(traj[-1, :, :3] - traj[0, :, :3], axis=1).max() < 2e-3
    assert np.abs(traj[-1, :, 7:13]).max() < 2e-2


def test_gpu_box_slides_down_incline():
    _cuda()
    theta, mu = 0.35, 0.1
    traj, sp = _incline_run(theta, mu, 90)
    d = np.array([-np.cos(theta), 0.0, -np.sin(theta)])
    v = traj[:, :, 7:10] @ d
    acc = (v[89] - v[30]) / (59 * sp.dt)
    expect = 9.81 * (np.sin(theta) - mu * np.cos(theta))
    assert np.abs(acc - expect).max() < 0.03 * expect + 0.05, (acc, expect)


def test_gpu_heightfield_can_be_removed():
    """set_heightfield(None) restores the flat plane: a box resting on a 1 m
    plateau falls back to z = 0.05."""
    _cuda()
    desc, sp, root, dof, props, pt, vt = pm.sim(pm.box_body(), n=2, dt=0.01, substeps=2)
    root[:, 0:3] = [[2.0, 2.0, 1.1], [3.0, 3.0, 1.1]]
    g = _gpu_sim(pm.box_body(), sp, 2, root, dof, props, pt, vt)
    g.set_heightfield(np.ones((20, 20), np.float32), 0.5, 1.0, 0.0, 0.0)
    for _ in range(100):
        g.simulate()
    z = g.root_state[:, 2].cpu().numpy()
    assert np.abs(z - 1.05).max() < 3e-3, z
    g.set_heightfield(None)
    for _ in range(150):
        g.simulate()
    z = g.root_state[:, 2].cpu().numpy()
    assert np.abs(z - 0.05).max() < 3e-3, z


def test_gpu_gogoro_terrain_step_matches_oracle_along_300_steps():
    """Gogoro with USE_TERAIN (gogoro_new.py:26,157-181,523-534): terrain
    spawn heights and wheel-terrain contact, teacher-forced against the oracle."""
    _cuda()
    from tests.gpu_harness import gogoro_terrain
    err = gogoro_terrain(num_envs=64, steps=300, seed=4)
    print(err)
    assert err["spawn_z_max"] > 0.05           # the envs really stand on raised terrain
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_terrain_free_running_matches_oracle():
    """Free-running fp32 GPU vs fp64 oracle on the Perlin terrain, at
    north_star's 1e-3.  The heightfield is piecewise planar, so a small state
    difference can put a tyre's support point on the other side of a triangle
    edge for one step (the contact normal jumps): round 3 measured a 1.26e-3
    spike on this seed (scripts/terrain_free_drift.py) and bounded the run at
    2e-3; since round 4's TGS conditioning fixes the run stays at 5e-5 (round
    5, profiles/r5/gpu_tests.log), so the bar is the strict one again.
    Resets must agree on every step, except a threshold tie: an
    env whose clean roll lies within 1e-3 of the 0.30 fall threshold may fall
    one step apart (seed 6, step 27: |roll| = 0.30 +- 4.5e-5); the comparison
    ends there, because the reset draws then desynchronise the streams."""
    _cuda()
    from tests.gpu_harness import gogoro_terrain
    err = gogoro_terrain(num_envs=64, steps=60, seed=6, forced=False)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] or err["ties_within_tol"], err
    assert err["compared_steps"] >= 25, err


def test_gpu_gogoro_terrain_forced_on_the_free_running_seed():
    """Teacher-forced (1e-3, north_star) on the seed of the free-running test."""
    _cuda()
    from tests.gpu_harness import gogoro_terrain
    err = gogoro_terrain(num_envs=64, steps=60, seed=6)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err

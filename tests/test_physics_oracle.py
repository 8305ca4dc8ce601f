"""Known-answer tests pinning the fp64 physics oracle (oracle/physics_ref.c).

PhysX itself is unavailable, so the oracle is pinned by
analytic results: free fall, pendulum period, torque-free rigid-body
invariants, momentum conservation of an internal-force chain, drive steady
states, joint limits, resting contact, Coulomb sliding.  CPU only."""
import numpy as np
import pytest

from tests import physics_models as pm
from tests.oracle_lib import physics_step
from thormang_isaacgym_amd.abi import (TG_PROP_DAMPING, TG_PROP_DRIVE_MODE, TG_PROP_EFFORT, TG_PROP_STIFFNESS,
                                       TG_PROP_VELOCITY)


def quat_to_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def run(state, steps, record=None):
    desc, sp, root, dof, props, pt, vt = state
    out = []
    for _ in range(steps):
        physics_step(desc, sp, root, dof, props, pt, vt)
        if record:
            out.append(record(root, dof))
    return np.array(out)


def test_free_fall_matches_semi_implicit_euler():
    st = pm.sim(pm.free_body(), dt=0.01, substeps=2)
    st[2][0, 2] = 10.0
    traj = run(st, 50, lambda r, d: (r[0, 2], r[0, 9]))
    h, g = 0.005, 9.81
    n = 2 * np.arange(1, 51)
    np.testing.assert_allclose(traj[:, 1], -g * h * n, rtol=1e-6)
    np.testing.assert_allclose(traj[:, 0], 10.0 - g * h * h * n * (n + 1) / 2, atol=1e-5)


def test_pendulum_small_angle_period():
    l, m, Ic = 0.5, 1.0, 0.01
    st = pm.pendulum(l, m, Ic)
    st = pm.sim(st, dt=0.001, substeps=1, fix_base_link=True)
    st[3][0, 0] = 0.05
    th = run(st, 5000, lambda r, d: d[0, 0])
    s = np.sign(th)
    cross = np.nonzero(s[1:] * s[:-1] < 0)[0]
    period = 2 * np.mean(np.diff(cross)) * 0.001
    T = 2 * np.pi * np.sqrt((Ic + m * l * l) / (m * 9.81 * l))
    assert abs(period - T) / T < 3e-3


def test_torque_free_body_conserves_momentum_and_energy():
    I = np.array([0.2, 0.5, 0.9])
    st = pm.sim(pm.free_body(tuple(I)), dt=0.001, substeps=1, gravity=(0, 0, 0))
    st[2][0, 10:13] = [1.0, 2.0, 0.5]
    st[2][0, 7:10] = [0.3, -0.1, 0.2]

    def rec(r, d):
        R = quat_to_R(r[0, 3:7].astype(np.float64))
        w = r[0, 10:13].astype(np.float64)
        Iw = R @ np.diag(I) @ R.T
        return np.concatenate([Iw @ w, [0.5 * w @ Iw @ w], r[0, 7:10]])

    tr = run(st, 2000, rec)
    L0 = tr[0, :3]
    assert np.abs(tr[:, :3] - L0).max() / np.linalg.norm(L0) < 2e-3
    assert np.abs(tr[:, 3] - tr[0, 3]).max() / tr[0, 3] < 2e-2
    np.testing.assert_allclose(tr[:, 4:7], np.tile([0.3, -0.1, 0.2], (len(tr), 1)), atol=1e-5)


def test_chain_internal_drive_keeps_system_com_fixed():
    """Zero gravity, no contact: an internal joint drive must not move the system COM."""
    m = pm.chain()
    st = pm.sim(m, dt=0.002, substeps=1, gravity=(0, 0, 0))
    desc, sp, root, dof, props, pt, vt = st
    props[TG_PROP_DRIVE_MODE, 0, 0] = 2
    props[TG_PROP_DAMPING, 0, 0] = 5.0
    props[TG_PROP_EFFORT, 0, 0] = 1e9
    vt[0, 0] = 4.0
    tr = run(st, 500, lambda r, d: np.concatenate([pm.system_com(m, r[0], d[:, 0]), d[:, 1]]))
    assert np.all(np.isfinite(tr))
    assert abs(tr[-1, 3] - 4.0) < 0.05          # drive reached its target rate
    assert np.abs(tr[:, :3] - tr[0, :3]).max() < 2e-3


def test_velocity_drive_steady_state_and_effort_limit():
    st = pm.sim(pm.pendulum(axis="0 0 1"), dt=0.01, substeps=2, fix_base_link=True)
    desc, sp, root, dof, props, pt, vt = st
    props[TG_PROP_DRIVE_MODE, 0, 0] = 2
    props[TG_PROP_DAMPING, 0, 0] = 1000.0
    props[TG_PROP_EFFORT, 0, 0] = 1e6
    vt[0, 0] = 7.0
    tr = run(st, 20, lambda r, d: d[0, 1])
    assert abs(tr[-1] - 7.0) < 1e-3
    # effort-limited: constant acceleration effort / I_pivot
    st = pm.sim(pm.pendulum(axis="0 0 1"), dt=0.01, substeps=2, fix_base_link=True)
    desc, sp, root, dof, props, pt, vt = st
    props[TG_PROP_DRIVE_MODE, 0, 0] = 2
    props[TG_PROP_DAMPING, 0, 0] = 1000.0
    props[TG_PROP_EFFORT, 0, 0] = 0.5
    vt[0, 0] = 100.0
    tr = run(st, 10, lambda r, d: d[0, 1])
    Ip = 0.01   # COM lies on the vertical axis: only the rotational inertia about z
    np.testing.assert_allclose(tr[-1], 0.5 / Ip * 0.1, rtol=2e-3)


def test_position_drive_converges():
    st = pm.sim(pm.pendulum(axis="0 0 1"), dt=0.01, substeps=2, fix_base_link=True)
    desc, sp, root, dof, props, pt, vt = st
    props[TG_PROP_DRIVE_MODE, 0, 0] = 1
    props[TG_PROP_STIFFNESS, 0, 0] = 3000.0
    props[TG_PROP_DAMPING, 0, 0] = 300.0
    props[TG_PROP_EFFORT, 0, 0] = 1e6
    pt[0, 0] = 0.4
    tr = run(st, 100, lambda r, d: d[0, 0])
    assert abs(tr[-1] - 0.4) < 1e-4


def test_joint_limit_holds_against_gravity():
    st = pm.sim(pm.pendulum(limits=(-0.3, 0.3)), dt=0.01, substeps=2, fix_base_link=True)
    st[3][0, 0] = 0.0
    # gravity swings the arm towards +-pi/2 around y; the limit must stop it
    st[2][0, 3:7] = [0, np.sin(0.7), 0, np.cos(0.7)]   # tilt the fixed base so gravity has a lever arm
    tr = run(st, 300, lambda r, d: d[0, 0])
    assert np.abs(tr).max() < 0.36
    assert abs(abs(tr[-1]) - 0.3) < 0.01


@pytest.mark.parametrize("shape", ["sphere", "box"])
def test_resting_contact(shape):
    m = pm.sphere_body(0.1) if shape == "sphere" else pm.box_body()
    st = pm.sim(m, dt=0.01, substeps=2)
    st[2][0, 2] = 0.3
    tr = run(st, 300, lambda r, d: r[0].copy())
    z_rest = 0.1 if shape == "sphere" else 0.05
    assert abs(tr[-1, 2] - z_rest) < 2e-3
    assert np.abs(tr[-1, 7:13]).max() < 1e-2
    assert tr[:, 2].min() > z_rest - 0.02   # no tunnelling


def test_coulomb_sliding_distance():
    mu = 0.5
    st = pm.sim(pm.box_body(mu=mu), dt=0.005, substeps=1, ground_friction=mu)
    st[2][0, 2] = 0.05
    st[2][0, 7] = 2.0
    tr = run(st, 200, lambda r, d: r[0, [0, 7]].copy())
    d_exp = 2.0 ** 2 / (2 * mu * 9.81)
    assert abs(tr[-1, 0] - d_exp) / d_exp < 0.05
    assert abs(tr[-1, 1]) < 1e-3

"""Rigid-body state tensor (acquire/refresh_rigid_body_state_tensor; SURVEY
§8b boundary): the oracle's link states checked by finite differences of the
forward kinematics (velocities are the time derivatives of the link com
positions and orientations), and the root-link row against the root state.
The GPU kernel is compared with the oracle in tests/test_gpu_physics.py."""
import numpy as np
import pytest

from tests.oracle_lib import rigid_body_states
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.sim import load_model


def quat_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def random_state(m, n, rs):
    root = np.zeros((n, 13), np.float32)
    root[:, :3] = rs.normal(0, 1, (n, 3))
    q = rs.normal(0, 1, (n, 4))
    root[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    root[:, 7:13] = rs.normal(0, 1, (n, 6))
    dof = np.zeros((n * m.num_dof, 2), np.float32)
    dof[:, 0] = rs.uniform(-1, 1, n * m.num_dof)
    dof[:, 1] = rs.normal(0, 1, n * m.num_dof)
    return root, dof


def advance(m, root, dof, dt):
    """Root pose and dof positions moved along the current velocities by dt (exact for the root rotation)."""
    r, d = root.astype(np.float64).copy(), dof.astype(np.float64).copy()
    n = r.shape[0]
    c0 = np.asarray(abi.model_arrays(m)["link_inertia"][0, 1:4], np.float64)
    for e in range(n):
        R = quat_R(r[e, 3:7])
        w = r[e, 10:13]
        v_origin = r[e, 7:10] - np.cross(w, R @ c0)
        r[e, :3] += dt * v_origin
        an = np.linalg.norm(w) * dt
        ax = w / max(np.linalg.norm(w), 1e-300)
        dq = np.concatenate([np.sin(an / 2) * ax, [np.cos(an / 2)]])
        x1, y1, z1, w1 = dq
        x2, y2, z2, w2 = r[e, 3:7]
        r[e, 3:7] = [w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2]
        # the com velocity of the root link is unchanged over the step for this kinematic check
    d[:, 0] += dt * d[:, 1]
    return r, d


@pytest.mark.parametrize("name", ["thormang", "gogoro"])
def test_oracle_link_velocities_are_fk_derivatives(name):
    m = load_model(name)
    desc = abi.ModelDesc(m)
    rs = np.random.default_rng(3)
    root, dof = random_state(m, 4, rs)
    out = rigid_body_states(desc, root, dof)
    assert out.shape == (4, m.num_bodies, 13)
    # root row = root state (quaternion up to sign)
    np.testing.assert_allclose(out[:, 0, :3], root[:, :3], atol=1e-6)
    sgn = np.sign(np.sum(out[:, 0, 3:7] * root[:, 3:7], axis=1, keepdims=True))
    np.testing.assert_allclose(out[:, 0, 3:7] * sgn, root[:, 3:7], atol=1e-6)
    np.testing.assert_allclose(out[:, 0, 7:13], root[:, 7:13], atol=1e-5)
    # central differences of link com positions and orientations
    h = 1e-3
    rp, dp = advance(m, root, dof, h)
    rm, dm = advance(m, root, dof, -h)
    op = rigid_body_states(desc, rp.astype(np.float32), dp.astype(np.float32)).astype(np.float64)
    om = rigid_body_states(desc, rm.astype(np.float32), dm.astype(np.float32)).astype(np.float64)
    com = np.asarray(abi.model_arrays(m)["link_inertia"][:, 1:4], np.float64)
    for e in range(4):
        for l in range(m.num_bodies):
            Rp, Rm = quat_R(op[e, l, 3:7]), quat_R(om[e, l, 3:7])
            cp = op[e, l, :3] + Rp @ com[l]
            cm = om[e, l, :3] + Rm @ com[l]
            np.testing.assert_allclose((cp - cm) / (2 * h), out[e, l, 7:10], atol=2e-2, rtol=2e-3,
                                       err_msg=f"{name} link {l} com velocity")
            Wx = (Rp - Rm) / (2 * h) @ quat_R(out[e, l, 3:7]).T     # dR/dt R^T = [w]x
            w = np.array([Wx[2, 1] - Wx[1, 2], Wx[0, 2] - Wx[2, 0], Wx[1, 0] - Wx[0, 1]]) / 2
            np.testing.assert_allclose(w, out[e, l, 10:13], atol=2e-2, rtol=2e-3,
                                       err_msg=f"{name} link {l} angular velocity")


def test_oracle_pendulum_link_position():
    """Fixed-base pendulum (kat model): the bob link's origin and com follow
    the joint angle analytically."""
    from tests import physics_models as pm
    m = pm.pendulum()
    desc = abi.ModelDesc(m)
    a = abi.model_arrays(m)
    root = np.zeros((1, 13), np.float32)
    root[0, 6] = 1
    dof = np.array([[0.7, 1.3]], np.float32)
    out = rigid_body_states(desc, root, dof)
    l = 1
    o = a["link_origin"][l]
    ax = a["link_axis"][l]
    R = o[:9].reshape(3, 3).astype(np.float64)
    from scipy.spatial.transform import Rotation
    Rj = Rotation.from_rotvec(0.7 * ax / np.linalg.norm(ax)).as_matrix()
    Rl = R @ Rj
    np.testing.assert_allclose(out[0, l, :3], o[9:12], atol=1e-6)
    np.testing.assert_allclose(quat_R(out[0, l, 3:7]), Rl, atol=1e-6)
    c = a["link_inertia"][l, 1:4]
    w = 1.3 * (R @ ax)
    np.testing.assert_allclose(out[0, l, 10:13], w, atol=1e-6)
    np.testing.assert_allclose(out[0, l, 7:10], np.cross(w, Rl @ c), atol=1e-6)

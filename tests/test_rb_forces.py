"""apply_rigid_body_force_tensors (reference call site
tasks/gogoro_realistic_turning_sim_paper.py:449-457): the reduction of
per-link forces / torques [N*L,3] to the step kernel's group wrenches.

CPU: the oracle's reduction (oracle/physics_ref.c
oracle_rigid_body_force_wrench) against an independent numpy evaluation built
on the oracle's link states, in both frames, plus the physical check that a
force on a body of a single-link group at its com is a pure force.  GPU: the
library's rb_force_kernel against the oracle (tests/test_gpu_physics.py)."""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import lib, ptr, rigid_body_states
from tests.test_rigid_body_states import quat_R, random_state
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.sim import load_model


def oracle_wrench(m, root, dof, forces, torques=None, space=0, mass_scale=None):
    n = root.shape[0]
    out = np.zeros((n, m.num_groups, 6), np.float32)
    desc = abi.ModelDesc(m)   # owns the arrays desc.desc points into: keep it alive over the call
    lib().oracle_rigid_body_force_wrench(C.byref(desc.desc), n, ptr(root), ptr(dof),
                                         ptr(mass_scale) if mass_scale is not None else None, ptr(forces),
                                         ptr(torques) if torques is not None else None, space, ptr(out))
    return out


def numpy_wrench(m, root, dof, forces, torques, space, mass_scale):
    n, L, G = root.shape[0], m.num_bodies, m.num_groups
    st = rigid_body_states(abi.ModelDesc(m), root, dof).astype(np.float64)
    desc = abi.ModelDesc(m).arrays
    mass = desc["link_inertia"][:, 0].astype(np.float64)
    com = desc["link_inertia"][:, 1:4].astype(np.float64)
    grp = np.asarray(desc["link_group"])
    out = np.zeros((n, G, 6))
    for e in range(n):
        R = np.stack([quat_R(st[e, l, 3:7]) for l in range(L)])
        pc = st[e, :, :3] + np.einsum("lij,lj->li", R, com)
        ml = mass * (mass_scale[e] if mass_scale is not None else 1.0)
        f = forces[e].astype(np.float64)
        t = np.zeros((L, 3)) if torques is None else torques[e].astype(np.float64)
        if space == 1:
            f, t = np.einsum("lij,lj->li", R, f), np.einsum("lij,lj->li", R, t)
        for g in range(G):
            ls = np.nonzero(grp == g)[0]
            cg = (ml[ls, None] * pc[ls]).sum(0) / ml[ls].sum()
            out[e, g, :3] = f[ls].sum(0)
            out[e, g, 3:] = (t[ls] + np.cross(pc[ls] - cg, f[ls])).sum(0)
    return out


@pytest.mark.parametrize("name", ["gogoro", "thormang"])
@pytest.mark.parametrize("space", [0, 1])
def test_oracle_reduction_matches_numpy(name, space):
    m = load_model(name)
    n, L = 6, m.num_bodies
    rs = np.random.default_rng(11 + space)
    root, dof = random_state(m, n, rs)
    f = rs.normal(0, 20.0, (n, L, 3)).astype(np.float32)
    t = rs.normal(0, 2.0, (n, L, 3)).astype(np.float32)
    ms = rs.uniform(0.9, 1.1, (n, L)).astype(np.float32)
    got = oracle_wrench(m, root, dof, f, t, space, ms)
    ref = numpy_wrench(m, root, dof, f, t, space, ms)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-4)


def test_force_at_com_of_single_link_group_is_pure_force():
    m = load_model("thormang")
    grp = np.asarray(abi.ModelDesc(m).arrays["link_group"])
    single = [l for l in range(m.num_bodies) if (grp == grp[l]).sum() == 1]
    assert single
    n = 3
    root, dof = random_state(m, n, np.random.default_rng(2))
    f = np.zeros((n, m.num_bodies, 3), np.float32)
    f[:, single[0]] = [3.0, -4.0, 5.0]
    out = oracle_wrench(m, root, dof, f)
    g = grp[single[0]]
    np.testing.assert_allclose(out[:, g, :3], np.broadcast_to([3.0, -4.0, 5.0], (n, 3)), atol=1e-6)
    np.testing.assert_allclose(out[:, g, 3:], 0.0, atol=1e-5)
    other = [k for k in range(m.num_groups) if k != g]
    assert np.abs(out[:, other]).max() == 0.0


def test_torque_only_and_total_force_conserved():
    m = load_model("gogoro")
    n, L = 4, m.num_bodies
    rs = np.random.default_rng(3)
    root, dof = random_state(m, n, rs)
    f = rs.normal(0, 5.0, (n, L, 3)).astype(np.float32)
    out = oracle_wrench(m, root, dof, f)
    np.testing.assert_allclose(out[..., :3].sum(1), f.sum(1), rtol=1e-5, atol=1e-4)
    t = rs.normal(0, 1.0, (n, L, 3)).astype(np.float32)
    out_t = oracle_wrench(m, root, dof, np.zeros_like(f), t)
    np.testing.assert_allclose(out_t[..., 3:].sum(1), t.sum(1), rtol=1e-5, atol=1e-4)

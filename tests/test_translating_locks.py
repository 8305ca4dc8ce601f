"""The Gogoro seat chain as translating locks (model/codegen.py
translating_locks; csrc/articulation_kernels.h tl_update): moving the locked
prismatic seat joints base_z -> base_x -> base_y only translates the rider,
so the fused epilogue updates the rider group's composite from stored mass
moments instead of re-composing the env.  CPU: the tables codegen emits, and
the moment-update algebra (restated in numpy) against a from-scratch
composite of the group's links at the new seat positions, both built on the
oracle's link kinematics."""
import numpy as np

from tests.oracle_lib import rigid_body_states
from tests.test_rigid_body_states import quat_R
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.model import codegen
from thormang_isaacgym_amd.sim import load_model


def test_codegen_finds_the_seat_chain_only_on_the_scooters_with_in_place_resets():
    m = load_model("gogoro")
    t = codegen.translating_locks(m, abi.ModelDesc(m).arrays)
    names = [m.links[l].name for l in t["tl_link"]]
    assert t["NTL"] == 3 and names == ["dummy_link1", "dummy_link2", "pelvis_link"]
    dn = m.dof_names
    assert [dn[d] for d in t["tl_dof"]] == ["base_z", "base_x", "base_y"]
    # the grip groups hang below the whole chain
    assert sorted(g for g, mask in t["ag"]) == [4, 5] and all(mask == 7 for _, mask in t["ag"])
    for name in ("thormang", "kat_chain"):
        mm = load_model(name)
        assert codegen.translating_locks(mm, abi.ModelDesc(mm).arrays)["NTL"] == 0
    # the paper's V12 scooter has the same chain (its resets move it in place too)
    v12 = load_model("gogoro_v12")
    assert codegen.translating_locks(v12, abi.ModelDesc(v12).arrays)["NTL"] == 3


def _group_links(m, a, g):
    return [l for l in range(m.num_bodies) if int(a["link_group"][l]) == g]


def _poses(m, q):
    """Link poses with the root at the origin (= the root group's frame)."""
    root = np.zeros((1, 13), np.float32)
    root[0, 6] = 1.0
    dof = np.zeros((m.num_dof, 2), np.float32)
    dof[:, 0] = q
    st = rigid_body_states(abi.ModelDesc(m), root, dof)[0].astype(np.float64)
    R = np.stack([quat_R(st[l, 3:7]) for l in range(m.num_bodies)])
    return R, st[:, :3]


def _composite(m, a, links, R, P):
    """Mass, com, inertia about the com (3x3) and the second moment about the
    origin (rotated link inertias included) of a set of links."""
    I6 = a["link_inertia"].astype(np.float64)
    mass, S, Io = 0.0, np.zeros(3), np.zeros((3, 3))
    for l in links:
        ml = I6[l, 0]
        Ic = np.array([[I6[l, 4], I6[l, 7], I6[l, 8]], [I6[l, 7], I6[l, 5], I6[l, 9]], [I6[l, 8], I6[l, 9], I6[l, 6]]])
        p = P[l] + R[l] @ I6[l, 1:4]
        mass += ml
        S += ml * p
        Io += R[l] @ Ic @ R[l].T + ml * (p @ p * np.eye(3) - np.outer(p, p))
    c = S / mass
    return mass, c, Io - mass * (c @ c * np.eye(3) - np.outer(c, c)), S, Io


def test_moment_update_equals_a_fresh_composite():
    m = load_model("gogoro")
    a = abi.ModelDesc(m).arrays
    t = codegen.translating_locks(m, a)
    g0 = t["tl_group"]
    links = _group_links(m, a, g0)
    rs = np.random.default_rng(3)
    q0 = np.zeros(m.num_dof)
    q0[t["tl_dof"]] = rs.normal(0, 0.02, 3)
    R0, P0 = _poses(m, q0)
    mass, _, _, S, Io = _composite(m, a, links, R0, P0)
    # per lock: moments of the links below it and its axis in the group frame
    mk, Sk, w = [], [], []
    I6 = a["link_inertia"].astype(np.float64)
    for k, lk in enumerate(t["tl_link"]):
        below = [l for l in links if (t["link_tl"][l] >> k) & 1]
        mk.append(sum(I6[l, 0] for l in below))
        Sk.append(sum(I6[l, 0] * (P0[l] + R0[l] @ I6[l, 1:4]) for l in below))
        par = int(a["link_parent"][lk])
        Ro = a["link_origin"][lk][:9].reshape(3, 3).astype(np.float64)
        w.append(R0[par] @ Ro @ a["link_axis"][lk].astype(np.float64))
    for trial in range(5):
        q1 = q0.copy()
        q1[t["tl_dof"]] = rs.normal(0, 0.02, 3)
        u = [(q1[d] - q0[d]) * w[k] for k, d in enumerate(t["tl_dof"])]
        S1 = S + sum(mk[k] * u[k] for k in range(3))
        Io1 = Io.copy()
        for k in range(3):
            Io1 += 2 * (Sk[k] @ u[k]) * np.eye(3) - np.outer(Sk[k], u[k]) - np.outer(u[k], Sk[k])
            for j in range(3):
                Io1 += mk[max(k, j)] * ((u[k] @ u[j]) * np.eye(3) - np.outer(u[k], u[j]))
        c1 = S1 / mass
        I1 = Io1 - mass * (c1 @ c1 * np.eye(3) - np.outer(c1, c1))
        R1, P1 = _poses(m, q1)
        mass_r, c_r, I_r, _, _ = _composite(m, a, links, R1, P1)
        assert abs(mass - mass_r) < 1e-9
        np.testing.assert_allclose(c1, c_r, atol=1e-6)
        np.testing.assert_allclose(I1, I_r, atol=2e-5 * np.abs(I_r).max())
        # the grip groups' joint placements move by the whole chain's shift
        for g, mask in t["ag"]:
            r = int(a["group_root"][g])
            par = int(a["link_parent"][r])
            to = a["link_origin"][r][9:12].astype(np.float64)
            t0, t1 = P0[par] + R0[par] @ to, P1[par] + R1[par] @ to
            np.testing.assert_allclose(t1, t0 + sum(u[k] for k in range(3) if (mask >> k) & 1), atol=1e-6)

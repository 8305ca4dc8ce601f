"""Small analytic articulations for the physics known-answer tests (CPU oracle
and GPU kernel alike).  Built from URDF text with the product's own URDF
loader, so the same model path is exercised."""
from __future__ import annotations

import numpy as np

from thormang_isaacgym_amd.abi import ModelDesc, default_dof_props, sim_params_from_cfg


from thormang_isaacgym_amd.model.kat_models import box_body, chain, free_body, pendulum, sphere_body, urdf_model  # noqa: F401


def sim(m, n=1, dt=0.01, substeps=1, gravity=(0, 0, -9.81), solver_type=0, **ao):
    sp = sim_params_from_cfg({"dt": dt, "substeps": substeps, "gravity": list(gravity),
                              "physx": {"rest_offset": 0.0, "max_depenetration_velocity": 1.0,
                                        "solver_type": solver_type}},
                             dict(dict(angular_damping=0.0, linear_damping=0.0, contact_iterations=16), **ao), n)
    desc = ModelDesc(m)
    D = m.num_dof
    props = default_dof_props(m, n)
    root = np.zeros((n, 13), np.float32)
    root[:, 6] = 1.0
    dof = np.zeros((n * D, 2), np.float32)
    pt = np.zeros((n, D), np.float32)
    vt = np.zeros((n, D), np.float32)
    return desc, sp, root, dof, props, pt, vt


def _rpy_free_R(o):
    return np.asarray(o, np.float64)


def system_com(m, root, q):
    """World COM of an articulation from the root state and dof positions (plain numpy FK)."""
    from thormang_isaacgym_amd.model.urdf import JOINT_PRISMATIC, JOINT_REVOLUTE
    x, y, z, w = [float(v) for v in root[3:7]]
    R0 = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    Rs, ps = [], []
    tot, acc = 0.0, np.zeros(3)
    for i, l in enumerate(m.links):
        if l.parent < 0:
            R, p = R0, np.asarray(root[0:3], np.float64)
        else:
            j = m.joints[l.joint]
            Ro, to = np.asarray(j.origin_rot), np.asarray(j.origin_pos, np.float64)
            a = np.asarray(j.axis)
            if j.jtype == JOINT_REVOLUTE:
                th = float(q[j.dof])
                K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
                Ro = Ro @ (np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K)
            elif j.jtype == JOINT_PRISMATIC:
                to = to + Ro @ a * float(q[j.dof])
            R, p = Rs[l.parent] @ Ro, ps[l.parent] + Rs[l.parent] @ to
        Rs.append(R)
        ps.append(p)
        acc += l.mass * (p + R @ np.asarray(l.com))
        tot += l.mass
    return acc / tot

"""Small analytic articulations for the physics known-answer tests (CPU oracle
and GPU kernel alike).  Built from URDF text with the product's own URDF
loader, so the same model path is exercised."""
from __future__ import annotations

import os
import tempfile

import numpy as np

from thormang_isaacgym_amd.abi import ModelDesc, default_dof_props, sim_params_from_cfg
from thormang_isaacgym_amd.model.urdf import Shape, load_urdf


def _inertial(m, com=(0, 0, 0), I=(0.1, 0.1, 0.1)):
    return (f'<inertial><origin xyz="{com[0]} {com[1]} {com[2]}"/><mass value="{m}"/>'
            f'<inertia ixx="{I[0]}" iyy="{I[1]}" izz="{I[2]}" ixy="0" ixz="0" iyz="0"/></inertial>')


def urdf_model(name, text, shapes=(), locked=()):
    with tempfile.NamedTemporaryFile("w", suffix=".urdf", delete=False) as f:
        f.write(f'<robot name="{name}">{text}</robot>')
        path = f.name
    try:
        m = load_urdf(path, name, extra_shapes=list(shapes))
    finally:
        os.unlink(path)
    m.build_groups(list(locked))
    return m


def free_body(I=(0.2, 0.5, 0.9), mass=2.0, shapes=()):
    return urdf_model("kat_free", f'<link name="b">{_inertial(mass, I=I)}</link>', shapes)


def pendulum(l=0.5, mass=1.0, Ic=0.01, axis="0 1 0", limits=None):
    lim = f'<limit lower="{limits[0]}" upper="{limits[1]}" effort="100" velocity="100"/>' if limits else \
        '<limit effort="100" velocity="100"/>'
    jt = "revolute" if limits else "continuous"
    return urdf_model("kat_pendulum",
                      f'<link name="base">{_inertial(1.0)}</link>'
                      f'<link name="arm">{_inertial(mass, (0, 0, -l), (Ic, Ic, Ic))}</link>'
                      f'<joint name="hinge" type="{jt}"><parent link="base"/><child link="arm"/>'
                      f'<origin xyz="0 0 1.0"/><axis xyz="{axis}"/>{lim}</joint>')


def chain():
    return urdf_model("kat_chain",
                      f'<link name="a">{_inertial(1.5, (0.1, 0, 0), (0.02, 0.05, 0.04))}</link>'
                      f'<link name="b">{_inertial(0.7, (0.2, 0.02, 0), (0.01, 0.03, 0.03))}</link>'
                      f'<link name="c">{_inertial(0.4, (0.1, 0, 0.03), (0.005, 0.01, 0.01))}</link>'
                      '<joint name="j1" type="continuous"><parent link="a"/><child link="b"/>'
                      '<origin xyz="0.3 0 0" rpy="0.1 0.2 0.3"/><axis xyz="0 0 1"/></joint>'
                      '<joint name="j2" type="prismatic"><parent link="b"/><child link="c"/>'
                      '<origin xyz="0.4 0 0"/><axis xyz="1 0 0"/><limit lower="-1" upper="1" effort="10" velocity="10"/></joint>')


def sphere_body(r=0.1, mass=1.0):
    return free_body((0.4 * mass * r * r,) * 3, mass,
                     [Shape("sphere", "b", [0, 0, 0], np.eye(3).tolist(), [r], 1.0)])


def box_body(half=(0.1, 0.075, 0.05), mass=2.0, mu=1.0):
    I = [mass / 3 * (half[1] ** 2 + half[2] ** 2), mass / 3 * (half[0] ** 2 + half[2] ** 2),
         mass / 3 * (half[0] ** 2 + half[1] ** 2)]
    return free_body(I, mass, [Shape("box", "b", [0, 0, 0], np.eye(3).tolist(), list(half), mu)])


def sim(m, n=1, dt=0.01, substeps=1, gravity=(0, 0, -9.81), **ao):
    sp = sim_params_from_cfg({"dt": dt, "substeps": substeps, "gravity": list(gravity),
                              "physx": {"rest_offset": 0.0, "max_depenetration_velocity": 1.0}},
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

"""Small analytic articulations used by the engine's known-answer tests
(tests/test_physics_oracle.py on the CPU oracle, tests/test_gpu_physics.py on
the HIP kernel).  They are compiled into libtgsim.so like the task models so
the GPU kernel can be checked on cases with closed-form answers."""
from __future__ import annotations

import os
import tempfile

import numpy as np

from .urdf import Shape, load_urdf


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


def free_body(I=(0.2, 0.5, 0.9), mass=2.0, shapes=(), name="kat_free"):
    return urdf_model(name, f'<link name="b">{_inertial(mass, I=I)}</link>', shapes)


def pendulum(l=0.5, mass=1.0, Ic=0.01, axis="0 1 0", limits=None, name=None):
    lim = f'<limit lower="{limits[0]}" upper="{limits[1]}" effort="100" velocity="100"/>' if limits else \
        '<limit effort="100" velocity="100"/>'
    jt = "revolute" if limits else "continuous"
    name = name or ("kat_pendulum_" + {"0 1 0": "y", "0 0 1": "z"}.get(axis, "a"))
    return urdf_model(name,
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
                     [Shape("sphere", "b", [0, 0, 0], np.eye(3).tolist(), [r], 1.0)], name="kat_sphere")


def box_body(half=(0.1, 0.075, 0.05), mass=2.0, mu=1.0):
    I = [mass / 3 * (half[1] ** 2 + half[2] ** 2), mass / 3 * (half[0] ** 2 + half[2] ** 2),
         mass / 3 * (half[0] ** 2 + half[1] ** 2)]
    return free_body(I, mass, [Shape("box", "b", [0, 0, 0], np.eye(3).tolist(), list(half), mu)], name="kat_box")



def all_models():
    """Default-parameter instances compiled into the library."""
    return [free_body(), pendulum(), pendulum(axis="0 0 1"), chain(), sphere_body(), box_body()]

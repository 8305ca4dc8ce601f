"""Compile the reference's assets into the build's JSON articulation models.

Runs in the build container only (reads /root/reference/assets); the JSON
output under ``model/compiled/`` is committed, so neither the GPU box nor the
product path needs the URDF files.

* ``gogoro``  -- ``assets/urdf/gogoro/urdf/scooter_V13.urdf`` exactly as the
  registered task loads it (tasks/gogoro_new.py:198-213).  Tyre collision
  meshes (``wheel_V3.obj``, ``<sdf resolution=1500>``, scooter_V13.urdf:1732-1768)
  become analytic tori fitted to the mesh profile; shape friction from
  gogoro_new.py:285-291 (rear 0.98, front 0.9).  The 0.1 m ``cam_link`` box
  (scooter_V13.urdf:1635) is dropped: the episode ends at |roll| >= 0.30 rad
  (gogoro_new.py:654,677) long before the rider's head can reach the ground.
  Locked joints: every ``joints_pos`` entry of cfg/task/Gogoro.yaml:61-93 plus
  the seat joints base_x/y/z (gogoro_new.py:257-262,562-572).
* ``gogoro_v12`` -- ``scooter_V12.urdf``, the asset of the unregistered "paper"
  variant (tasks/gogoro_realistic_turning_sim_paper.py:203): same joint tree and
  tyres as V13, different link inertias.
* ``thormang`` -- ``assets/urdf/gogoro/urdf/thormang3.urdf`` (44 links, 33
  revolute DOFs) for the walk task, which the reference does not contain
  (SURVEY.md §8 a11).  That URDF carries placeholder inertias (1.0 kg m^2 on
  every link) and no collision geometry; we take the mesh-derived inertias
  scooter_V13.urdf holds for the same links and the foot boxes of
  ``thormang3/thormang3.structure.leg.xacro:242-250`` (0.22 x 0.15 x 0.015 m,
  offset (0, +-0.014, -0.02) in the foot link).
* ``thormang_wb`` -- the same humanoid with whole-body contact for the limbs
  that reach the ground in a kneel or a fall: besides the foot boxes, the shin
  boxes (``thormang3.structure.leg.xacro:135-138``, 0.11 x 0.16 x 0.33 m at
  (0.01, -+0.065, -0.145) in the knee-pitch link) and the hand boxes
  (``thormang3.structure.arm.xacro:252-254``, 0.07 x 0.1 x 0.06 m at
  (0.07, +-0.045, 0) in the wrist-pitch link).  Selected by the walk cfg's
  ``env.asset.wholeBodyCollision`` (tasks/thormang_walk.py).
"""
from __future__ import annotations

import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from thormang_isaacgym_amd.model.urdf import Shape, load_urdf, _parse_inertial  # noqa: E402

ASSETS = "/root/reference/assets/urdf/gogoro"

GOGORO_LOCKED = [
    "l_arm_el_y", "l_arm_wr_r", "head_y", "r_arm_grip", "l_arm_wr_p", "torso_y", "r_arm_sh_r", "l_arm_sh_p1",
    "l_arm_sh_r", "l_leg_an_r", "l_leg_an_p", "r_leg_hip_p", "r_leg_an_p", "l_arm_wr_y", "l_leg_hip_p",
    "r_leg_hip_y", "l_leg_hip_r", "l_leg_kn_p", "r_arm_sh_p2", "r_arm_sh_p1", "l_leg_hip_y", "r_leg_hip_r",
    "l_arm_sh_p2", "r_arm_wr_y", "head_p", "r_arm_wr_p", "r_arm_wr_r", "r_arm_el_y", "l_arm_grip", "r_leg_an_r",
    "r_leg_kn_p", "base_x", "base_y", "base_z",
]


def build_gogoro(urdf="scooter_V13.urdf", name="gogoro"):
    m = load_urdf(f"{ASSETS}/urdf/{urdf}", name, mesh_root=f"{ASSETS}/meshes",
                  shape_friction={"back": 0.98, "front": 0.9})
    m.shapes = [s for s in m.shapes if s.kind == "torus"]
    m.build_groups(GOGORO_LOCKED)
    return m


def build_thormang(whole_body=False):
    v13 = ET.parse(f"{ASSETS}/urdf/scooter_V13.urdf").getroot()
    override = {}
    for l in v13.findall("link"):
        el = l.find("inertial")
        if el is not None:
            override[l.get("name")] = _parse_inertial(el)[2]
    eye = [[1, 0, 0], [0, 1, 0], [0, 0, 1]]
    shapes = [Shape("box", "l_leg_foot_link", [0.0, 0.014, -0.02], eye, [0.11, 0.075, 0.0075], 1.0),
              Shape("box", "r_leg_foot_link", [0.0, -0.014, -0.02], eye, [0.11, 0.075, 0.0075], 1.0)]
    if whole_body:   # shins (leg xacro :135-138, :410-413) and hands (arm xacro :252-254, :604-606), half sizes
        shapes += [Shape("box", "l_leg_kn_p_link", [0.01, -0.065, -0.145], eye, [0.055, 0.08, 0.165], 1.0),
                   Shape("box", "r_leg_kn_p_link", [0.01, 0.065, -0.145], eye, [0.055, 0.08, 0.165], 1.0),
                   Shape("box", "l_arm_wr_p_link", [0.07, 0.045, 0.0], eye, [0.035, 0.05, 0.03], 1.0),
                   Shape("box", "r_arm_wr_p_link", [0.07, -0.045, 0.0], eye, [0.035, 0.05, 0.03], 1.0)]
    m = load_urdf(f"{ASSETS}/urdf/thormang3.urdf", "thormang_wb" if whole_body else "thormang",
                  inertia_override=override, extra_shapes=shapes)
    m.build_groups([])
    return m


def main():
    out = os.path.join(HERE, "compiled")
    os.makedirs(out, exist_ok=True)
    from thormang_isaacgym_amd.model.kat_models import all_models
    # gogoro_v12: the asset of the "paper" variant (tasks/gogoro_realistic_turning_sim_paper.py:203;
    # same tree as V13, different link inertias), same locks (cfg/task/Gogoro_paper.yaml joints_pos)
    for m in [build_gogoro(), build_gogoro("scooter_V12.urdf", "gogoro_v12"), build_thormang(),
              build_thormang(whole_body=True)] + all_models():
        with open(os.path.join(out, f"{m.name}.json"), "w") as f:
            f.write(m.to_json())
        print(m.name, "links", m.num_bodies, "dofs", m.num_dof, "groups", m.num_groups, "active", len(m.active_dofs),
              "shapes", len(m.shapes))


if __name__ == "__main__":
    main()

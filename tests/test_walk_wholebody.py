"""Whole-body contact for the humanoid (model ``thormang_wb``, selected by
``env.asset.wholeBodyCollision``): the xacro's shin and hand boxes collide
besides the feet (model/build_models.py).  CPU: the model and its kernel
layout, and the oracle's kneel-and-fall -- with the foot boxes alone the
pelvis sinks through the floor, with the whole body it stays up."""
import os
import re

import numpy as np

from tests.gpu_harness import NumpyDraws, OracleWalk, walk_kneel_cfg

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(os.path.dirname(HERE), "thormang_isaacgym_amd", "csrc", "generated")


def test_wholebody_model_carries_the_xacro_shin_and_hand_boxes():
    from thormang_isaacgym_amd.sim import load_model
    from thormang_isaacgym_amd.tasks.thormang_walk import walk_model_name
    m = load_model("thormang_wb")
    links = sorted(s.link for s in m.shapes)
    assert links == sorted(["l_leg_foot_link", "r_leg_foot_link", "l_leg_kn_p_link", "r_leg_kn_p_link",
                            "l_arm_wr_p_link", "r_arm_wr_p_link"])
    shin = [s for s in m.shapes if s.link == "l_leg_kn_p_link"][0]
    assert shin.kind == "box" and np.allclose(shin.params, [0.055, 0.08, 0.165]) and np.allclose(shin.pos, [0.01, -0.065, -0.145])
    base = load_model("thormang")
    assert [l.name for l in m.links] == [l.name for l in base.links] and m.dof_names == base.dof_names
    assert walk_model_name(walk_kneel_cfg(4)) == "thormang_wb"
    assert walk_model_name(walk_kneel_cfg(4, whole_body=False)) == "thormang"
    # 42 contact rows (6 boxes x (4 normals + 3 friction)): 8 envs per workgroup fit the LDS
    txt = open(os.path.join(GEN, "Model_thormang_wb.inc")).read()
    assert re.search(r"NROWS = 42\b", txt) and re.search(r"EPB = 8\b", txt)
    assert re.search(r"EPB = 16\b", open(os.path.join(GEN, "Model_thormang.inc")).read())


def _kneel(whole_body, n=8, steps=150):
    o = OracleWalk(walk_kneel_cfg(n, whole_body), NumpyDraws(0))
    zs = []
    for _ in range(steps):
        o.step(np.zeros((n, o.D), np.float32))
        zs.append(o.a["root"][:, 2].copy())
    return np.array(zs)


def test_oracle_kneel_rests_on_shins_and_hands_only_with_the_whole_body():
    feet, wb = _kneel(False), _kneel(True)
    assert feet.min() < -0.3, feet.min()      # foot boxes alone: the pelvis goes through the floor
    assert wb.min() > 0.15, wb.min()          # shins and hands hold it up
    assert np.isfinite(wb).all()

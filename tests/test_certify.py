"""CPU tests of the teacher-forced harness's discontinuity certificate
(tests/gpu_harness.certify_discontinuity): a GPU-vs-oracle disagreement is
excused only when the fp64 oracle itself lands on the GPU's result from
inputs moved by about one fp32 ulp.

Fixture tests/golden/walk_gate_outlier.npz: one env-step of the 16384-env
ThormangWalkDR teacher-forced run (torch seed 0, step 56, env 15805),
captured on the MI355X by scripts/dev/r6_walk_outlier.py -- the physics
inputs after the pre-physics and the GPU's root after the step, 0.159 from
the unperturbed oracle (a foot corner 1e-8 m inside the contact gate takes
0.48 N s; outside it, none)."""
import os

import numpy as np

from tests.gpu_harness import NumpyDraws, OracleWalk, certify_discontinuity, walk_cfg

FIX = os.path.join(os.path.dirname(__file__), "golden", "walk_gate_outlier.npz")


def _oracle_with(c):
    orc = OracleWalk(walk_cfg(1, "ThormangWalkDR", dr=True), NumpyDraws(0), threads=1)
    orc.props[:, 0, :] = c["props"]
    orc._pin = {"root": c["root"][None].copy(), "dof": c["dof"].copy(), "pos_target": c["pos_target"][None].copy(),
                "force": c["force"][None].copy(),
                "dr": {"mass_scale": c["mass_scale"][None].copy(), "mu": c["mu"][None].copy(),
                       "gravity": c["gravity"].copy()}}
    return orc


def test_gate_outlier_is_certified():
    c = dict(np.load(FIX))
    orc = _oracle_with(c)
    d0 = float(np.abs(orc.replay_env(0, c["root"], c["dof"]) - c["gpu_root"]).max())
    assert d0 > 0.1                       # the unperturbed oracle is far from the GPU
    ok, dist = certify_discontinuity(orc, 0, c["gpu_root"])
    assert ok and dist < 1e-3, (ok, dist)


def test_agreeing_or_unexplained_results_are_not_certified():
    c = dict(np.load(FIX))
    orc = _oracle_with(c)
    own = orc.replay_env(0, c["root"], c["dof"])
    assert certify_discontinuity(orc, 0, own) == (False, 0.0)       # no disagreement to excuse
    wrong = own.copy()
    wrong[7:10] += 0.05                                              # a jump no replay produces
    ok, dist = certify_discontinuity(orc, 0, wrong)
    assert not ok and dist > 1e-3

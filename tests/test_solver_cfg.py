"""Solver cfg semantics: every ``sim.physx`` key of the
reference cfgs (``isaacgymenvs/cfg/task/Gogoro.yaml:15-28``, set on PhysX's
params by ``tasks/base/vec_task.py:470-482``) either changes the simulated
result or raises a ``SolverCfgWarning`` naming it.  CPU only: the result
check runs the oracle engine (oracle/physics_ref.c), which reads the same
``tg_sim_params`` the HIP kernel does."""
import warnings

import numpy as np
import pytest
import yaml

from tests import physics_models as pm
from tests.oracle_lib import physics_step
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.abi import ModelDesc, SolverCfgWarning, default_dof_props, sim_params_from_cfg

GOGORO_YAML = "thormang_isaacgym_amd/cfg/task/Gogoro.yaml"


def _cfg_sim():
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, GOGORO_YAML)) as f:
        return yaml.safe_load(f)["sim"]


def test_gogoro_cfg_warns_on_each_unhonoured_key():
    with pytest.warns(SolverCfgWarning) as rec:
        sim_params_from_cfg(_cfg_sim())
    msg = " ".join(str(w.message) for w in rec)
    for k in ("solver_type", "num_velocity_iterations", "contact_offset", "bounce_threshold_velocity"):
        assert k in msg, k
    # resource knobs and honoured keys are not reported
    for k in ("num_threads", "num_subscenes", "max_gpu_contact_pairs", "num_position_iterations", "rest_offset",
              "max_depenetration_velocity"):
        assert f"{k}:" not in msg, k


def test_honoured_keys_do_not_warn():
    physx = {"solver_type": 0, "num_position_iterations": 6, "num_velocity_iterations": 0, "rest_offset": 0.0,
             "max_depenetration_velocity": 1.0, "num_threads": 4, "use_gpu": True}
    with warnings.catch_warnings():
        warnings.simplefilter("error", SolverCfgWarning)
        sp = sim_params_from_cfg({"dt": 0.01, "physx": physx})
    assert sp.contact_iterations == 6


def test_unknown_key_is_reported():
    assert "friction_offset_threshold" in abi.unhonoured_physx_keys({"friction_offset_threshold": 0.04})


def _drop_tilted_box(physx, steps=40):
    m = pm.box_body(mu=0.8)
    sp = sim_params_from_cfg({"dt": 0.01, "substeps": 2, "gravity": [0, 0, -9.81], "physx": physx},
                             dict(angular_damping=0.0, linear_damping=0.0, ground_friction=0.8), 1, warn=False)
    desc = ModelDesc(m)
    props = default_dof_props(m, 1)
    root = np.zeros((1, 13), np.float32)
    c, s = np.cos(0.15), np.sin(0.15)
    root[0, 2] = 0.06
    root[0, 3:7] = [s, 0.0, 0.0, c]          # tilted 0.3 rad about x
    root[0, 7] = 0.7                          # sliding while it lands
    dof = np.zeros((0, 2), np.float32)
    pt = np.zeros((1, 0), np.float32)
    vt = np.zeros((1, 0), np.float32)
    for _ in range(steps):
        physics_step(desc, sp, root, dof, props, pt, vt)
    return root[0].copy()


BASE = {"num_position_iterations": 8, "rest_offset": 0.0, "max_depenetration_velocity": 1.0}


@pytest.mark.parametrize("key,value", [("num_position_iterations", 1), ("rest_offset", 0.01),
                                       ("max_depenetration_velocity", 0.05)])
def test_honoured_key_changes_the_result(key, value):
    a = _drop_tilted_box(BASE)
    b = _drop_tilted_box(dict(BASE, **{key: value}))
    assert np.abs(a - b).max() > 1e-5, (key, a, b)

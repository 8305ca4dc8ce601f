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


@pytest.mark.parametrize("task", ["Gogoro", "GogoroPaper", "ThormangWalk", "ThormangWalkDR"])
def test_task_cfgs_raise_no_solver_warning(task):
    """Every sim.physx key of the shipped task cfgs is honoured or inert since
    round 5 (contact_offset was the last one): building
    the sim params from them raises no SolverCfgWarning."""
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "thormang_isaacgym_amd", "cfg", "task", task + ".yaml")) as f:
        sim = yaml.safe_load(f)["sim"]
    with warnings.catch_warnings():
        warnings.simplefilter("error", SolverCfgWarning)
        sp = sim_params_from_cfg(sim)
    assert abs(sp.contact_offset - float(sim["physx"]["contact_offset"])) < 1e-9
    assert sp.solver_type == 1


def test_solver_type_mapping():
    assert sim_params_from_cfg({"dt": 0.01, "physx": {}}, warn=False).solver_type == 1   # IsaacGym's default: TGS
    assert sim_params_from_cfg({"dt": 0.01, "physx": {"solver_type": 0}}, warn=False).solver_type == 0
    assert "solver_type" in abi.unhonoured_physx_keys({"solver_type": 2})
    assert "solver_type" not in abi.unhonoured_physx_keys({"solver_type": 1})


def test_honoured_keys_do_not_warn():
    physx = {"solver_type": 0, "num_position_iterations": 6, "num_velocity_iterations": 3, "rest_offset": 0.0,
             "max_depenetration_velocity": 1.0, "num_threads": 4, "use_gpu": True}
    with warnings.catch_warnings():
        warnings.simplefilter("error", SolverCfgWarning)
        sp = sim_params_from_cfg({"dt": 0.01, "physx": physx})
    assert sp.contact_iterations == 6 and sp.velocity_iterations == 3
    # IsaacGym's default of one velocity iteration when the key is absent
    assert sim_params_from_cfg({"dt": 0.01, "physx": {}}, warn=False).velocity_iterations == 1


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


@pytest.mark.parametrize("solver", [0, 1])
@pytest.mark.parametrize("key,value", [("num_position_iterations", 1), ("num_velocity_iterations", 0),
                                       ("rest_offset", 0.01), ("max_depenetration_velocity", 0.05)])
def test_honoured_key_changes_the_result(key, value, solver):
    a = _drop_tilted_box(dict(BASE, solver_type=solver))
    b = _drop_tilted_box(dict(BASE, solver_type=solver, **{key: value}))
    assert np.abs(a - b).max() > 1e-5, (key, a, b)


def test_solver_type_changes_the_result():
    a = _drop_tilted_box(dict(BASE, solver_type=0))
    b = _drop_tilted_box(dict(BASE, solver_type=1))
    assert np.abs(a - b).max() > 1e-5, (a, b)


def _push_out(viters, steps=1, solver=0, depth=0.004, vz=0.0, baumgarte=0.5):
    """A box resting ``depth`` INSIDE the ground (negative: above it) moving
    at ``vz``: the biased sweeps push it out."""
    m = pm.box_body(mu=0.8)
    physx = {"num_position_iterations": 8, "num_velocity_iterations": viters, "rest_offset": 0.0,
             "max_depenetration_velocity": 10.0, "solver_type": solver}
    sp = sim_params_from_cfg({"dt": 0.01, "substeps": 1, "gravity": [0, 0, 0], "physx": physx},
                             dict(angular_damping=0.0, linear_damping=0.0, ground_friction=0.8,
                                  baumgarte=baumgarte), 1, warn=False)
    desc = ModelDesc(m)
    props = default_dof_props(m, 1)
    root = np.zeros((1, 13), np.float32)
    root[0, 2] = 0.05 - depth   # box half height 0.05 (kat_models.box_body) - depth
    root[0, 6] = 1.0
    root[0, 9] = vz
    z0 = float(root[0, 2])
    dof = np.zeros((0, 2), np.float32)
    z = np.zeros((1, 0), np.float32)
    for _ in range(steps):
        physics_step(desc, sp, root, dof, props, z, z)
    return z0, root[0].copy()


def test_velocity_iterations_drop_the_push_out_from_the_stored_velocity():
    """num_velocity_iterations (PhysX semantics, Gogoro.yaml:21): the position
    still moves by the biased sweeps' push-out velocity, but the velocity the
    step stores is the bias-free one -- the penetration is recovered without
    leaving the box flying up.  Without velocity sweeps the push-out velocity
    is stored."""
    z0, r0 = _push_out(0)
    z1, r1 = _push_out(16)
    assert r0[2] > z0 + 1e-4 and abs(r1[2] - r0[2]) < 1e-7   # same push-out of the position
    assert r0[9] > 0.05                                        # biased: push-out velocity stored
    assert abs(r1[9]) < 1e-6 and np.abs(r1[10:13]).max() < 1e-6   # bias-free: nothing stored
    # Gauss-Seidel: fewer sweeps remove the stored push-out only in part (the
    # corner rows are solved one after another), monotonically
    v = [abs(_push_out(k)[1][9]) for k in (1, 4, 8)]
    assert r0[9] > v[0] > v[1] > v[2] > abs(r1[9])


def test_tgs_sub_steps_recover_more_of_the_penetration():
    """solver_type 1 (TGS): the 8 position iterations are sub-steps of h/8,
    each re-forming the push-out target from the separation its predecessors
    left, so one step recovers about 1 - (1 - baumgarte)^8 of a 4 mm
    penetration where the PGS's converged push-out recovers baumgarte of it;
    the positions move by the mean sub-step velocity, and the velocity
    iterations leave nothing stored."""
    z0, rp = _push_out(16, solver=0)
    _, rt = _push_out(16, solver=1)
    dp, dt = rp[2] - z0, rt[2] - z0
    assert 0.0019 < dp < 0.0021                   # PGS: baumgarte x depth
    # TGS: most of it; one Gauss-Seidel sweep per sub-step over the 4 coupled
    # corner rows overshoots the rest offset by a few per cent at most
    assert 0.0035 < dt < 0.0042, dt
    assert abs(rt[9]) < 1e-6 and np.abs(rt[10:13]).max() < 1e-6


def test_tgs_speculative_landing_stores_no_approach_velocity():
    """A box 1 mm above the ground falling at 1 m/s (one 10 ms substep):
    both solvers stop it at the ground over the step, but the PGS stores the
    speculative approach velocity -(gap)/h while TGS's last sub-step has
    reached the ground and stores (almost) none."""
    z0, rp = _push_out(0, solver=0, depth=-0.001, vz=-1.0)
    _, rt = _push_out(0, solver=1, depth=-0.001, vz=-1.0)
    for r in (rp, rt):
        assert abs((r[2] - z0) + 0.001) < 2e-4, r[2] - z0   # moved down by about the gap
    assert abs(rp[9] + 0.1) < 1e-3, rp[9]                   # PGS: -gap/h stored
    assert abs(rt[9]) < 0.02, rt[9]                         # TGS: at rest at the ground


def test_tgs_velocity_iterations_warm_start_from_the_mean_and_stop_the_landing():
    """With velocity iterations TGS warm-starts them from the sub-steps' mean
    multipliers (DESIGN.md §2 "TGS conditioning"): the box of the landing
    above is still stopped at the ground over the step, and the bias-free
    sweeps (targets over h from the final separation, about 0) remove the
    approach velocity the mean carries."""
    z0, r = _push_out(4, solver=1, depth=-0.001, vz=-1.0)
    assert abs((r[2] - z0) + 0.001) < 2e-4, r[2] - z0
    assert abs(r[9]) < 0.02, r[9]


@pytest.mark.parametrize("solver,viters,rest", [(1, 1, 0.0), (1, 4, 0.002), (0, 1, 0.0), (0, 0, 0.0)])
def test_landing_known_answer_no_rebound_and_rest_height(solver, viters, rest):
    """A physics known answer for the restated TGS / PGS contact solve,
    independent of the oracle-vs-kernel comparison (the TGS
    target and warm-start choices of round 4 are this restatement's, so
    GPU-vs-oracle agreement cannot show they are physical): a box dropped
    0.2 m onto the ground with the walk cfg's step (dt 1/60 x 2, 4 position
    iterations) lands without rebound and rests at half height + rest offset
    (tests/physics_models.landing_checks; the GPU kernel is held to the same
    answer in tests/test_gpu_physics.py).  Every shipped cfg runs at least
    one velocity iteration (Gogoro 4, the walk 1); TGS with none stores the
    last sub-step's push-out velocity (PhysX's own semantics without
    velocity iterations: a resting box keeps +3.5 mm/s stored at a constant
    height), which test_tgs_without_velocity_iterations_stores_the_bias pins."""
    zs, vs = pm.drop_box(solver, viters=viters, rest_offset=rest)
    r = pm.landing_checks(zs, vs, rest_offset=rest)
    assert r["ok"], r


def test_tgs_without_velocity_iterations_stores_the_bias():
    """TGS with num_velocity_iterations 0: the stored velocity is the last
    position sub-step's, which carries the push-out bias, so a resting box
    keeps a small upward velocity while its height stays put (what PhysX
    documents velocity iterations for); with one velocity iteration it is
    gone.  Recorded so a change of this semantics is seen."""
    z0, v0 = pm.drop_box(1, viters=0, steps=120)
    z1, v1 = pm.drop_box(1, viters=1, steps=120)
    assert abs(z0[-1] - z0[-20]) < 1e-6 and 1e-3 < v0[-1] < 1e-2, (z0[-1], v0[-1])
    assert abs(v1[-1]) < 1e-3, v1[-1]


@pytest.mark.parametrize("solver", [0, 1])
def test_rows_on_a_fixed_base_take_no_impulse(solver):
    """A shape on a fixed base has no contact response (its Delassus diagonal
    is 0): its rows must take no impulse rather than divide by zero -- a
    fixed-base torso pushed 3 cm into the ground stays where it is, its legs
    swing, everything finite
    (round 5: the 1/W of such rows made every state NaN, in the oracle and
    the kernel, for any fixed-base model with a shape on its root)."""
    m = pm.jit_walker()   # a box torso (the root) on two legs
    desc, sp, root, dof, props, pt, vt = pm.sim(m, n=2, dt=0.01, substeps=2, solver_type=solver, fix_base_link=True)
    root[:, 2] = 0.02   # the torso box's half height is 0.05: 3 cm into the plane
    r0 = root.copy()
    for _ in range(5):
        physics_step(desc, sp, root, dof, props, pt, vt)
    assert np.isfinite(root).all() and np.isfinite(dof).all()
    np.testing.assert_array_equal(root, r0)
    assert np.abs(dof[:, 1]).max() > 0   # the legs swing under gravity


def test_contact_offset_default_follows_the_vec_task_base():
    """without a sim.physx.contact_offset key the default is the one
    the reference's base class leaves -- IsaacGym's 0.02 under
    vec_task.VecTask (Gogoro), 0.016 under multi_vec_task.MA_VecTask
    (multi_vec_task.py:322, the walk's MA_OP3 template); no asset option
    overrides it."""
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.tasks.base.vec_task import VecTask
    from thormang_isaacgym_amd.tasks.thormang_walk import ThormangWalk
    sim = {"dt": 0.01, "substeps": 1, "physx": {}}
    assert VecTask.default_contact_offset == 0.02 and ThormangWalk.default_contact_offset == 0.016
    sp = abi.sim_params_from_cfg(sim, {"contact_offset": 0.5}, 1, warn=False)
    assert abs(sp.contact_offset - 0.02) < 1e-9
    sp = abi.sim_params_from_cfg(sim, {}, 1, warn=False, default_contact_offset=ThormangWalk.default_contact_offset)
    assert abs(sp.contact_offset - 0.016) < 1e-9


@pytest.mark.parametrize("solver", [0, 1])
def test_contact_offset_known_answers(solver):
    """the contact_offset gate checked against what it must do, not
    against the kernel (both restate the same rule), PhysX's pair rule (a
    contact while the separation is below the shape's plus the plane's
    offset): a resting gap beyond it is free flight, exactly; a fast approach
    from inside it lands without tunnelling; the same approach from beyond it
    gets no row in its first substep (no CCD), then comes back to rest
    (tests/physics_models.contact_offset_checks; GPU twin in
    tests/test_gpu_physics.py)."""
    r = pm.contact_offset_checks(solver_type=solver)
    assert abs(r["rest_gap_dz"]) < 1e-7 and abs(r["rest_gap_dvz"]) < 1e-6, r   # (the state is stored in fp32)
    assert r["free_flight_z1"] < -0.01, r                     # without a row it would end below the ground
    assert r["fast_min_z"] > -0.002 and r["fast_z1"] > -0.002, r
    assert r["fast_vz1"] > -0.5 and abs(r["fast_final"]) < 1e-3, r
    assert r["beyond_min_z"] < -0.003, r                      # passed the surface in the row-less substep
    assert abs(r["beyond_final"]) < 2e-3 and abs(r["beyond_vz_final"]) < 0.05, r

"""HIP articulation kernel vs the fp64 oracle on the known-answer models, plus
the analytic checks themselves on the GPU (free fall, drive steady state,
resting contact, Coulomb sliding)."""
import numpy as np
import pytest
import torch

from tests import physics_models as pm
from tests.oracle_lib import physics_step
from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_DRIVE_MODE, TG_PROP_EFFORT, TG_PROP_STIFFNESS

pytestmark = pytest.mark.gpu


from tests.physics_models import jit_walker  # noqa: E402  (the run-time URDF's model)


def gpu_sim(model, sp, n, root, dof, props, pt, vt):
    from thormang_isaacgym_amd.sim import Sim
    s = Sim(model, sp, n, "cuda:0")
    s.root_state.copy_(torch.from_numpy(root))
    s.dof_state.copy_(torch.from_numpy(dof))
    s.dof_props.copy_(torch.from_numpy(props))
    s.dof_pos_target.copy_(torch.from_numpy(pt))
    s.dof_vel_target.copy_(torch.from_numpy(vt))
    s.env_dirty.fill_(1)
    return s


def side_by_side(model, steps, n=16, seed=0, setup=None, **simkw):
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    st = pm.sim(model, n=n, **simkw)
    desc, sp, root, dof, props, pt, vt = st
    rs = np.random.default_rng(seed)
    if setup:
        setup(rs, root, dof, props, pt, vt)
    g = gpu_sim(model, sp, n, root, dof, props, pt, vt)
    worst = 0.0
    for _ in range(steps):
        physics_step(desc, sp, root, dof, props, pt, vt)
        g.simulate()
        gr = g.root_state.cpu().numpy()
        gd = g.dof_state.cpu().numpy()
        scale = max(1.0, float(np.abs(root).max()))
        worst = max(worst, _maxerr(gr, root) / scale)
        if dof.size:
            worst = max(worst, _maxerr(gd, dof) / scale)
    return worst, g, root, dof


def _maxerr(a, b):
    """max |a - b|, inf when either side is not finite (a NaN would otherwise
    vanish in max(), and a run where both sides blow up would pass)"""
    if not (np.isfinite(a).all() and np.isfinite(b).all()):
        return float("inf")
    return float(np.abs(a - b).max())


def _spin(rs, root, dof, props, pt, vt):
    root[:, 2] = 1.0
    root[:, 7:10] = rs.normal(0, 1, (root.shape[0], 3))
    root[:, 10:13] = rs.normal(0, 2, (root.shape[0], 3))


@pytest.mark.parametrize("name", ["free", "chain", "pendulum"])
def test_gpu_matches_oracle_on_kat_models(name):
    if name == "free":
        m, kw, setup = pm.free_body(), dict(dt=0.01, substeps=2), _spin
    elif name == "chain":
        m, kw = pm.chain(), dict(dt=0.005, substeps=1, gravity=(0, 0, -9.81))

        def setup(rs, root, dof, props, pt, vt):
            _spin(rs, root, dof, props, pt, vt)
            dof[:, 1] = rs.normal(0, 2, dof.shape[0])
    else:
        m, kw = pm.pendulum(), dict(dt=0.01, substeps=2, fix_base_link=True)

        def setup(rs, root, dof, props, pt, vt):
            dof[:, 0] = rs.uniform(-1, 1, dof.shape[0])
            props[TG_PROP_DRIVE_MODE, :, 0] = 1
            props[TG_PROP_STIFFNESS, :, 0] = 50.0
            props[TG_PROP_DAMPING, :, 0] = 5.0
            props[TG_PROP_EFFORT, :, 0] = 1e9
            pt[:, 0] = rs.uniform(-0.5, 0.5, pt.shape[0])
    worst, *_ = side_by_side(m, 100, setup=setup, **kw)
    print({"model": name, "worst_state_err": worst})
    assert worst < 1e-3, worst


@pytest.mark.parametrize("solver", [0, 1])
@pytest.mark.parametrize("shape", ["sphere", "box"])
def test_gpu_contact_matches_oracle_and_rests(shape, solver):
    """Bodies dropped onto the plane, 200 free-running steps, under PGS
    (solver_type 0) and TGS (1: the 16 position iterations as sub-steps)."""
    m = pm.sphere_body(0.1) if shape == "sphere" else pm.box_body()

    def setup(rs, root, dof, props, pt, vt):
        root[:, 2] = rs.uniform(0.12, 0.4, root.shape[0])
        root[:, 7:9] = rs.normal(0, 0.5, (root.shape[0], 2))

    worst, g, root, dof = side_by_side(m, 200, setup=setup, dt=0.01, substeps=2, solver_type=solver)
    z_rest = 0.1 if shape == "sphere" else 0.05
    gr = g.root_state.cpu().numpy()
    print({"shape": shape, "solver": solver, "worst_state_err": worst, "rest_err": float(np.abs(gr[:, 2] - z_rest).max())})
    assert np.abs(gr[:, 2] - z_rest).max() < 3e-3
    assert worst < 1e-3, worst


@pytest.mark.parametrize("solver,viters,rest", [(1, 1, 0.0), (1, 4, 0.002), (0, 1, 0.0)])
def test_gpu_landing_known_answer_no_rebound_and_rest_height(solver, viters, rest):
    """The landing known answer of tests/test_solver_cfg.py on the GPU kernel
    itself (behaviour the physics requires, not agreement with the
    oracle): the box dropped 0.2 m with the walk cfg's step lands without
    rebound and rests at half height + rest offset."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    sims = {}

    def gpu_step(desc, sp, root, dof, props, pt, vt):
        if "g" not in sims:
            sims["g"] = gpu_sim(pm.box_body(mu=0.8), sp, 1, root, dof, props, pt, vt)
        g = sims["g"]
        g.simulate()
        root[...] = g.root_state.cpu().numpy()
    zs, vs = pm.drop_box(solver, viters=viters, rest_offset=rest, step_fn=gpu_step)
    r = pm.landing_checks(zs, vs, rest_offset=rest)
    print(r)
    assert r["ok"], r


@pytest.mark.parametrize("solver", [0, 1])
def test_gpu_contact_offset_known_answers(solver):
    """The contact_offset known answers of tests/test_solver_cfg.py on the GPU
    kernel (PhysX's pair rule): a resting gap beyond 2 x the offset
    is exact free flight; a 6 m/s approach from inside it lands without
    tunnelling; from beyond it, passes the surface in one substep and
    recovers."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")

    def make_step():
        sims = []

        def gpu_step(desc, sp, root, dof, props, pt, vt):
            if not sims:
                sims.append(gpu_sim(pm.box_body(mu=0.8), sp, 1, root, dof, props, pt, vt))
            sims[0].simulate()
            root[...] = sims[0].root_state.cpu().numpy()
        return gpu_step

    g = pm.contact_offset_checks(make_step, solver_type=solver)
    print({"gpu": g, "oracle": pm.contact_offset_checks(solver_type=solver)})
    assert abs(g["rest_gap_dz"]) < 1e-6 and abs(g["rest_gap_dvz"]) < 1e-5, g
    assert g["fast_min_z"] > -0.002 and g["fast_z1"] > -0.002, g
    assert g["fast_vz1"] > -0.5 and abs(g["fast_final"]) < 1e-3, g
    assert g["beyond_min_z"] < -0.003, g
    assert abs(g["beyond_final"]) < 2e-3 and abs(g["beyond_vz_final"]) < 0.05, g


def test_gpu_free_fall_exact():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    st = pm.sim(pm.free_body(), n=4, dt=0.01, substeps=2)
    desc, sp, root, dof, props, pt, vt = st
    root[:, 2] = 10.0
    g = gpu_sim(pm.free_body(), sp, 4, root, dof, props, pt, vt)
    for _ in range(50):
        g.simulate()
    r = g.root_state.cpu().numpy()
    n = 100
    h = 0.005
    np.testing.assert_allclose(r[:, 9], -9.81 * h * n, rtol=1e-5)
    np.testing.assert_allclose(r[:, 2], 10.0 - 9.81 * h * h * n * (n + 1) / 2, atol=1e-4)


@pytest.mark.parametrize("name", ["thormang", "gogoro"])
def test_gpu_rigid_body_states_match_oracle(name):
    """refresh_rigid_body_state_tensor (tg_rigid_body_states) vs the oracle's
    link states on random root / dof states."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    from tests.oracle_lib import rigid_body_states
    from tests.test_rigid_body_states import random_state
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.sim import Sim, load_model
    m = load_model(name)
    n = 256
    root, dof = random_state(m, n, np.random.default_rng(5))
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1, "gravity": [0, 0, -9.81]}, {}, n)
    s = Sim(m, sp, n, "cuda:0")
    s.root_state.copy_(torch.from_numpy(root))
    s.dof_state.copy_(torch.from_numpy(dof))
    rb = s.acquire_rigid_body_state_tensor()
    s.refresh_rigid_body_state_tensor()
    g = rb.view(n, m.num_bodies, 13).cpu().numpy()
    o = rigid_body_states(abi.ModelDesc(m), root, dof)
    sgn = np.sign(np.sum(g[..., 3:7] * o[..., 3:7], axis=-1, keepdims=True))
    np.testing.assert_allclose(g[..., :3], o[..., :3], atol=3e-5)
    np.testing.assert_allclose(g[..., 3:7] * sgn, o[..., 3:7], atol=3e-5)
    np.testing.assert_allclose(g[..., 7:13], o[..., 7:13], atol=2e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["thormang", "gogoro"])
@pytest.mark.parametrize("space", [0, 1])
def test_gpu_rigid_body_force_tensors_match_oracle(name, space):
    """apply_rigid_body_force_tensors (tg_apply_rigid_body_force_tensors, the
    reference's [N*L,3] layout, gogoro_realistic_turning_sim_paper.py:457) vs
    the oracle's reduction to group wrenches, on random states, forces,
    torques and per-env mass scales; then torques only."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    from tests.test_rb_forces import oracle_wrench
    from tests.test_rigid_body_states import random_state
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.sim import Sim, load_model
    m = load_model(name)
    n, L = 512, m.num_bodies
    rs = np.random.default_rng(21 + space)
    root, dof = random_state(m, n, rs)
    # locked joints at the centre of their windows, as the composite holds them
    # (the world-frame reduction takes its moment arms from the composite)
    props0 = abi.default_dof_props(m, 1)
    for d in m.locked_dofs:
        dof.reshape(n, -1, 2)[:, d, 0] = 0.5 * (props0[abi.TG_PROP_LOWER, 0, d] + props0[abi.TG_PROP_UPPER, 0, d])
    f = rs.normal(0, 20.0, (n, L, 3)).astype(np.float32)
    t = rs.normal(0, 2.0, (n, L, 3)).astype(np.float32)
    ms = rs.uniform(0.9, 1.1, (n, L)).astype(np.float32)
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1, "gravity": [0, 0, -9.81]}, {}, n)
    s = Sim(m, sp, n, "cuda:0")
    s.root_state.copy_(torch.from_numpy(root))
    s.dof_state.copy_(torch.from_numpy(dof))
    ids = torch.arange(n, device="cuda:0")
    s.set_body_mass_scale_indexed(torch.from_numpy(ms).cuda(), ids)
    # the reduction runs in the next simulate, from the state it starts at:
    # first inside that simulate's compose launch (the mass scales make every
    # env dirty), then -- nothing dirty -- by its own kernel
    ft, tt = torch.from_numpy(f).cuda().reshape(-1, 3), torch.from_numpy(t).cuda().reshape(-1, 3)
    for case in ("forces+torques", "torques only"):
        r0 = s.root_state.cpu().numpy().copy()
        d0 = s.dof_state.cpu().numpy().copy()
        if case == "forces+torques":
            assert s.apply_rigid_body_force_tensors(ft, tt, space)
            ref = oracle_wrench(m, r0, d0, f, t, space, ms)
            scale = np.abs(ref).max()
        else:
            assert s.apply_rigid_body_force_tensors(None, tt, space)
            ref = oracle_wrench(m, r0, d0, np.zeros_like(f), t, space, ms)
        s.simulate()
        torch.cuda.synchronize()
        np.testing.assert_allclose(s.body_force.cpu().numpy(), ref, atol=2e-5 * scale, rtol=1e-4, err_msg=case)


def test_gpu_runtime_loaded_model_matches_oracle():
    """gym.load_asset of a URDF that is not compiled in: Sim compiles its
    kernels at run time (tg_model_jit, hipRTC) and the GPU trajectory -- a
    hanging two-legged body, hips and a knee on PD drives, the other knee
    locked, joint limits -- matches the oracle over 150 steps."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.sim import compiled_model_hashes
    m = jit_walker()
    assert abi.ModelDesc(m).hash not in compiled_model_hashes()
    dl = m.dof_name_to_id()

    def setup(rs, root, dof, props, pt, vt):
        n = root.shape[0]
        root[:, 2] = 1.0
        for j in ("l_hip", "r_hip", "l_knee"):
            d = dl[j]
            props[TG_PROP_DRIVE_MODE, :, d] = 1
            props[TG_PROP_STIFFNESS, :, d] = 60.0
            props[TG_PROP_DAMPING, :, d] = 4.0
            props[TG_PROP_EFFORT, :, d] = 30.0
            pt[:, d] = rs.uniform(-1.0, 1.0, n)
        k = dl["r_knee"]
        props[4, :, k] = 0.3            # lock window [0.3, 0.3 + 1e-4]
        props[5, :, k] = 0.3001
        dof.reshape(n, -1, 2)[:, k, 0] = 0.30005
        dof.reshape(n, -1, 2)[:, dl["r_hip"], 1] = rs.normal(0, 2, n)

    worst, g, _, dof = side_by_side(m, 150, n=32, setup=setup, dt=0.01, substeps=2, fix_base_link=True)
    assert g.jit, "expected a run-time specialisation"
    moved = float(np.abs(dof.reshape(32, -1, 2)[:, dl["l_hip"], 0]).max())
    print({"runtime_model_worst_state_err": worst, "l_hip_max_abs_q": moved})
    assert moved > 0.05, moved          # the drives moved the legs (the comparison is not of a still body)
    assert worst < 1e-3, worst


@pytest.mark.parametrize("name", ["kat_box", "thormang"])
def test_gpu_runtime_specialisation_equals_compiled(name):
    """The run-time (hipRTC) specialisation of a compiled-in model, registered
    under another hash, against the compiled-in kernels on identical inputs:
    the box exercises the contact rows / PGS, the Thormang tree 16 lanes per
    env and ~150 KB of dynamic LDS through hipModuleLaunchKernel."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    from thormang_isaacgym_amd.sim import Sim, load_model
    m = load_model(name)
    n = 64
    kw = dict(dt=0.01, substeps=2) if name == "kat_box" else dict(dt=1 / 60, substeps=2, fix_base_link=True)
    desc, sp, root, dof, props, pt, vt = pm.sim(m, n=n, **kw)
    rs = np.random.default_rng(4)
    if name == "kat_box":
        root[:, 2] = rs.uniform(0.06, 0.3, n)
        root[:, 7:9] = rs.normal(0, 0.8, (n, 2))
        root[:, 10:13] = rs.normal(0, 2.0, (n, 3))
    else:
        root[:, 2] = 1.2
        dof[:, 0] = rs.uniform(-0.3, 0.3, dof.shape[0])
    sims = []
    for jh in (None, 0x7E57_0000_0000_0000 | (abi_hash(m) & 0xFFFF_FFFF)):
        s = Sim(m, sp, n, "cuda:0", jit_hash=jh)
        s.root_state.copy_(torch.from_numpy(root))
        s.dof_state.copy_(torch.from_numpy(dof))
        s.dof_props.copy_(torch.from_numpy(props))
        s.env_dirty.fill_(1)
        sims.append(s)
    assert not sims[0].jit and sims[1].jit
    for _ in range(60):
        for s in sims:
            s.simulate()
    torch.cuda.synchronize()
    for k in ("root_state", "dof_state"):
        a, b = getattr(sims[0], k), getattr(sims[1], k)
        if a.numel() == 0:   # the box has no dofs
            continue
        assert torch.isfinite(a).all()
        d = float((a - b).abs().max())
        assert d <= 1e-5, (k, d)


def abi_hash(m):
    from thormang_isaacgym_amd import abi
    return abi.ModelDesc(m).hash


def test_gpu_native_urdf_load_through_the_c_abi_alone():
    """gym.load_asset without the Python host: tg_model_load (csrc/model_load.cpp
    parses the URDF, builds the descriptor and the specialisation's traits and
    compiles them with hipRTC) of a URDF that is not compiled in -- every joint
    type, a locked joint, box / sphere / fitted-tyre shapes -- then a sim on
    the library's own descriptor, against the fp64 oracle on the Python host's
    parse of the same file (identical arrays: tests/test_model_load.py)."""
    import os
    from thormang_isaacgym_amd.sim import NativeModel, Sim, load_asset
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    here = os.path.dirname(os.path.abspath(__file__))
    urdf, meshes = os.path.join(here, "golden", "urdf", "loader_tree.urdf"), os.path.join(here, "golden", "urdf")
    nm = NativeModel(urdf, locked=["j_seat"], mesh_root=meshes)
    m = load_asset(urdf, locked=["j_seat"], mesh_root=meshes)
    n = 16
    desc, sp, root, dof, props, pt, vt = pm.sim(m, n=n, dt=0.01, substeps=2)
    assert nm.hash == desc.hash and nm.jit
    rs = np.random.default_rng(7)
    root[:, 2] = 1.5                                     # clear of the ground: free fall + joint dynamics
    root[:, 7:10] = rs.normal(0, 0.5, (n, 3))
    root[:, 10:13] = rs.normal(0, 1.0, (n, 3))
    dof[:, 1] = rs.normal(0, 1.0, dof.shape[0])
    props[TG_PROP_DRIVE_MODE] = 1                        # position drives on every dof
    props[TG_PROP_STIFFNESS] = 20.0
    props[TG_PROP_DAMPING] = 1.0
    props[TG_PROP_EFFORT] = 50.0
    g = Sim(nm, sp, n, "cuda:0")
    g.root_state.copy_(torch.from_numpy(root))
    g.dof_state.copy_(torch.from_numpy(dof))
    g.dof_props.copy_(torch.from_numpy(props))
    g.env_dirty.fill_(1)
    g.refresh()
    worst = 0.0
    for _ in range(40):
        physics_step(desc, sp, root, dof, props, pt, vt)
        g.simulate()
        worst = max(worst, _maxerr(g.root_state.cpu().numpy(), root), _maxerr(g.dof_state.cpu().numpy(), dof))
    print({"native_urdf_worst_state_err": worst})
    assert np.isfinite(worst) and worst < 1e-3, worst


def test_gpu_solver_type_switches_at_runtime():
    """gym.set_sim_params (tg_set_sim_params) switches the contact solve
    between PGS (solver_type 0) and TGS (1) from the next simulate on: boxes
    landing with some penetration, teacher-forced, each step against the
    oracle under the solver it ran (pose 1e-4, velocity 5e-3, as the contact
    tests), and the two solvers give different results from one state."""
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    m = pm.box_body()
    n = 16
    desc, sp, root, dof, props, pt, vt = pm.sim(m, n=n, dt=0.01, substeps=2)
    rs = np.random.default_rng(3)
    root[:, 2] = rs.uniform(0.046, 0.06, n)          # half height 0.05: some start 4 mm inside
    root[:, 7:9] = rs.normal(0, 0.5, (n, 2))
    root[:, 9] = -0.5
    g = gpu_sim(m, sp, n, root, dof, props, pt, vt)
    after = {}
    for solver in (0, 1, 0, 1, 1, 0):
        spg = g.get_sim_params()
        spg.solver_type = solver
        g.set_sim_params(spg)
        so = type(sp).from_buffer_copy(sp)
        so.solver_type = solver
        r = g.root_state.cpu().numpy().copy()
        d = g.dof_state.cpu().numpy().copy()
        r0 = r.copy()
        physics_step(desc, so, r, d, props, pt, vt)
        g.simulate()
        gr = g.root_state.cpu().numpy()
        print({"solver": solver, "pose_err": float(np.abs(gr[:, :7] - r[:, :7]).max()),
               "vel_err": float(np.abs(gr[:, 7:] - r[:, 7:]).max())})
        assert _maxerr(gr[:, :7], r[:, :7]) < 1e-4, solver
        assert _maxerr(gr[:, 7:], r[:, 7:]) < 1e-3, solver
        after.setdefault(solver, (r0, gr.copy()))
    # the same start state under the other solver differs
    r0, g0 = after[0]
    so = type(sp).from_buffer_copy(sp)
    so.solver_type = 1
    r1 = r0.copy()
    physics_step(desc, so, r1, dof.copy(), props, pt, vt)
    assert np.abs(r1[:, 7:] - g0[:, 7:]).max() > 1e-3

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
        worst = max(worst, float(np.abs(gr - root).max()) / scale)
        if dof.size:
            worst = max(worst, float(np.abs(gd - dof).max()) / scale)
    return worst, g, root, dof


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
    assert worst < 2e-3, worst


@pytest.mark.parametrize("shape", ["sphere", "box"])
def test_gpu_contact_matches_oracle_and_rests(shape):
    m = pm.sphere_body(0.1) if shape == "sphere" else pm.box_body()

    def setup(rs, root, dof, props, pt, vt):
        root[:, 2] = rs.uniform(0.12, 0.4, root.shape[0])
        root[:, 7:9] = rs.normal(0, 0.5, (root.shape[0], 2))

    worst, g, root, dof = side_by_side(m, 200, setup=setup, dt=0.01, substeps=2)
    z_rest = 0.1 if shape == "sphere" else 0.05
    gr = g.root_state.cpu().numpy()
    assert np.abs(gr[:, 2] - z_rest).max() < 3e-3
    assert worst < 5e-3, worst


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
    f = rs.normal(0, 20.0, (n, L, 3)).astype(np.float32)
    t = rs.normal(0, 2.0, (n, L, 3)).astype(np.float32)
    ms = rs.uniform(0.9, 1.1, (n, L)).astype(np.float32)
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1, "gravity": [0, 0, -9.81]}, {}, n)
    s = Sim(m, sp, n, "cuda:0")
    s.root_state.copy_(torch.from_numpy(root))
    s.dof_state.copy_(torch.from_numpy(dof))
    ids = torch.arange(n, device="cuda:0")
    s.set_body_mass_scale_indexed(torch.from_numpy(ms).cuda(), ids)
    assert s.apply_rigid_body_force_tensors(torch.from_numpy(f).cuda().reshape(-1, 3),
                                            torch.from_numpy(t).cuda().reshape(-1, 3), space)
    torch.cuda.synchronize()
    got = s.body_force.cpu().numpy()
    ref = oracle_wrench(m, root, dof, f, t, space, ms)
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got, ref, atol=2e-5 * scale, rtol=1e-4)
    s.apply_rigid_body_force_tensors(None, torch.from_numpy(t).cuda(), space)
    torch.cuda.synchronize()
    ref_t = oracle_wrench(m, root, dof, np.zeros_like(f), t, space, ms)
    np.testing.assert_allclose(s.body_force.cpu().numpy(), ref_t, atol=2e-5 * scale, rtol=1e-4)

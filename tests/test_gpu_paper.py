"""GPU parity for the Gogoro "paper" variant through the C-ABI.

* the three reference fixtures (tests/golden/make_golden_paper.py) are replayed
  through the product class -- recorded physics states and recorded draws
  injected -- so the HIP task kernels are compared with the reference module;
* the full env (task kernels + HIP articulation step, fixed and free base) runs
  beside the oracle env (oracle/gogoro_paper_task.c + fp64 physics) on
  identical draws.
"""
import contextlib
import os

import numpy as np
import pytest
import torch
from tests.gpu_harness import within
from tests.gpu_harness import maxerr

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


@contextlib.contextmanager
def switches(sw):
    from thormang_isaacgym_amd.tasks import gogoro_paper as gp
    saved = gp.current_switches()
    for k, v in sw.items():
        setattr(gp, k, v)
    try:
        yield gp
    finally:
        for k, v in saved.items():
            setattr(gp, k, v)


@pytest.mark.parametrize("name", ["paper_steps.npz", "paper_falls.npz", "paper_steps_flags.npz"])
def test_gpu_paper_kernels_replay_reference(name):
    _cuda()
    from tests.paper_harness import fixture_cfg, switches_from
    from thormang_isaacgym_amd.tasks.gogoro_draws import RecordedDraws
    f = np.load(os.path.join(GOLDEN, name))
    src = RecordedDraws(f["draw_kind"], f["draw_size"], f["draw_vals"])
    state = {"t": 0}
    cfg = fixture_cfg(f)
    cfg["sim"]["use_gpu_pipeline"] = True     # fixture cfg was recorded for the reference's CPU pipeline
    with switches(switches_from(f["flags"])) as gp:
        class Replay(gp.Gogoro):
            draw_source = src
            env_spacing = 0.0

            def simulate(self):
                t = state["t"]
                self.root_tensor.copy_(torch.from_numpy(f["sim_root"][t]))
                self.state_dof.copy_(torch.from_numpy(f["sim_dof"][t]))
                self.frame_count += 1

        env = Replay(cfg, "cuda:0", "cuda:0", -1, True, False, False)
    assert src.i == int(f["init_n_draws_init"])
    np.testing.assert_allclose(env.root_tensor.cpu().numpy(), f["init_root"], atol=1e-6)
    np.testing.assert_array_equal(env.state_dof.cpu().numpy(), f["init_dof"])
    err = 0.0
    for t in range(f["actions"].shape[0]):
        state["t"] = t
        obs, rew, reset, extras = env.step(torch.from_numpy(f["actions"][t]).cuda())
        assert src.i == int(f["draw_end"][t])
        np.testing.assert_array_equal(reset.cpu().numpy(), f["reset"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(extras["time_outs"].cpu().numpy(), f["time_outs"][t])
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), f["progress"][t])
        np.testing.assert_allclose(obs["obs"].cpu().numpy(), f["obs"][t], atol=2e-5, err_msg=f"obs step {t}")
        np.testing.assert_allclose(rew.cpu().numpy(), f["rew"][t], atol=2e-5, err_msg=f"rew step {t}")
        np.testing.assert_allclose(env.sim.dof_pos_target.cpu().numpy(), f["pos_target"][t], atol=1e-7)
        np.testing.assert_array_equal(env.sim.dof_vel_target.cpu().numpy(), f["vel_target"][t])
        for k in ("curent_command", "command_history", "yaw_command", "curent_speed", "steer_offsets",
                  "curent_speed_offset", "curent_imu_x_offset", "buffer_obs", "buffer_obs_noisy"):
            np.testing.assert_allclose(getattr(env, k).cpu().numpy(), f[k][t], atol=2e-5, err_msg=f"{k} {t}")
        np.testing.assert_array_equal(env.steer_delay.cpu().numpy(), f["steer_delay"][t])
        np.testing.assert_allclose(env.head_perturbation.cpu().numpy(), f["perturbation"][t], atol=2e-5)
        np.testing.assert_allclose(env.root_tensor.cpu().numpy(), f["root_after"][t], atol=1e-6)
        err = max(err, maxerr(obs["obs"].cpu().numpy(), f["obs"][t]))
    assert src.i == len(f["draw_kind"])
    print(name, "max obs err", err)


def _env_vs_oracle(sw, n=64, steps=80, seed=3, forced=False):
    from tests.gpu_harness import NumpyDraws
    from tests.paper_harness import OraclePaper
    from thormang_isaacgym_amd.cfg import load_task_cfg
    from thormang_isaacgym_amd.tasks.gogoro_cfg import env_origins
    cfg = load_task_cfg("GogoroPaper", num_envs=n)
    cfg["env"]["max_steps"] = 60
    cfg["noises"]["speed_freq_update"] = cfg["noises"]["yaw_freq_update"] = 25
    with switches(sw) as gp:
        class Env(gp.Gogoro):
            draw_source = NumpyDraws(seed)
        env = Env(cfg, "cuda:0", "cuda:0", -1, True, False, False)
        full = dict(gp.current_switches())
    orc = OraclePaper(load_task_cfg("GogoroPaper", num_envs=n) | {"env": cfg["env"], "noises": cfg["noises"]},
                      NumpyDraws(seed), full, root_origins=env_origins(n, 1.0))
    # the rounding control (fp32 oracle build) when the cfg asks for TGS (tests.gpu_harness.within)
    from tests.gpu_harness import tgs_configured
    ctl = OraclePaper(load_task_cfg("GogoroPaper", num_envs=n) | {"env": cfg["env"], "noises": cfg["noises"]},
                      NumpyDraws(seed), full, root_origins=env_origins(n, 1.0),
                      precision="f32") if tgs_configured(cfg) else None
    rs = np.random.default_rng(seed + 7)
    if forced:
        from tests.gpu_harness import forced_step_errors
        return forced_step_errors(env, orc, lambda o: rs.uniform(-1, 1, (n, 1)).astype(np.float32), steps, ctl=ctl)
    err = {"obs": 0.0, "rew": 0.0, "reset_equal": True, "timeout_equal": True, "resets": 0, "root": 0.0, "dof": 0.0}
    if ctl is not None:
        err["obs_f32"] = err["rew_f32"] = 0.0
    for t in range(steps):
        act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
        od, rew, reset, ex = env.step(torch.from_numpy(act).cuda())
        orc.pre(act[:, 0])
        orc.physics()
        o_obs, o_rew, o_reset, o_to = orc.post()
        if ctl is not None:
            ctl.pre(act[:, 0])
            ctl.physics()
            c_obs, c_rew = ctl.post()[:2]
            err["obs_f32"] = max(err["obs_f32"], maxerr(c_obs, o_obs))
            err["rew_f32"] = max(err["rew_f32"], maxerr(c_rew, o_rew))
        err["obs"] = max(err["obs"], maxerr(od["obs"].cpu().numpy(), o_obs))
        err["rew"] = max(err["rew"], maxerr(rew.cpu().numpy(), o_rew))
        err["reset_equal"] &= bool(np.array_equal(reset.cpu().numpy(), o_reset))
        err["timeout_equal"] &= bool(np.array_equal(ex["time_outs"].cpu().numpy().astype(np.uint8), o_to))
        err["resets"] += int(o_reset.sum())
        # the whole simulated state too, not only what the observations see
        # (round 5: a fixed-base wheel ran away unseen by obs and reward)
        err["root"] = max(err["root"], maxerr(env.sim.root_state.cpu().numpy(), orc.a["root"]))
        err["dof"] = max(err["dof"], maxerr(env.sim.dof_state.cpu().numpy()[:, 0], orc.a["dof_state"][:, 0]))
    return err


def test_gpu_paper_env_matches_oracle_fixed_base():
    """As committed (DEBUG = True): fixed base, pushes, start speed, 2-step steering delay."""
    _cuda()
    err = _env_vs_oracle({})
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    assert err["root"] < 1e-3 and err["dof"] < 1e-3, err   # the joints too (a wheel ran away unseen, round 5)


def test_gpu_paper_fixed_base_free_running_1000_steps():
    """north_star's horizon free-running on the paper variant's committed
    configuration (fixed base): 1000 steps with an episode reset every 60,
    pushes, command resamples every 25 and the 2-step steering delay."""
    _cuda()
    err = _env_vs_oracle({}, steps=1000)
    print(err)
    assert err["resets"] >= 64 * 16, err     # every env re-spawned along the way
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    assert err["root"] < 1e-3 and err["dof"] < 1e-3, err


FLIPPED = dict(DEBUGFIXBASE=False, USE_STEER_DELAY=True, RANDOM_DAMPING=True, CENTER_ROBOT=False)


def test_gpu_paper_env_matches_oracle_free_base_flags_flipped():
    """Free base, per-env steering delay, random steering damping, random seat
    offsets, pushes; random actions make the scooters fall, and the reward's
    tanh(50 x^2) terms amplify fp32-vs-fp64 drift, so the free-running horizon
    is 25 steps and the long horizon is teacher-forced below."""
    _cuda()
    err = _env_vs_oracle(FLIPPED, steps=25)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err
    assert err["root"] < 1e-3 and err["dof"] < 1e-3, err


def test_gpu_paper_free_base_step_matches_oracle_along_300_steps():
    _cuda()
    err = _env_vs_oracle(FLIPPED, steps=300, forced=True)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_paper_2048_envs_run():
    _cuda()
    import thormang_isaacgym_amd as tia
    env = tia.make(seed=3, task="GogoroPaper", num_envs=2048, sim_device="cuda:0", rl_device="cuda:0")
    assert env.obs_buf.shape == (2048, 160) and env.num_actions == 1
    g = torch.Generator(device="cuda:0").manual_seed(5)
    for _ in range(120):
        obs, rew, reset, extras = env.step(torch.rand(2048, 1, device="cuda:0", generator=g) * 2 - 1)
    assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    assert torch.isfinite(env.root_tensor).all()
    assert float(env.head_perturbation.abs().max()) > 0.0   # pushes happened


def test_gpu_paper_fused_step_equals_separate_calls(monkeypatch):
    """tg_paper_step (the pre-physics inside the step kernel, which also forms
    reward term 7's per-env partials, and a post launch that sums the batch
    itself) against the three separate calls (TG_PAPER_UNFUSED=1: post kernel
    partials, finish launch): the same operations in the same order, so every
    buffer agrees bit for bit -- including the head pushes, which tg_paper_step
    reduces inside its post launch, after a root write between two steps
    (the pre-reduced wrenches then give way to the next simulate's reduction)."""
    _cuda()
    import thormang_isaacgym_amd as tia
    out = []
    for unfused in ("0", "1"):
        monkeypatch.setenv("TG_PAPER_UNFUSED", unfused)
        env = tia.make(seed=11, task="GogoroPaper", num_envs=256, sim_device="cuda:0", rl_device="cuda:0")
        g = torch.Generator(device="cuda:0").manual_seed(9)
        ids = torch.arange(0, 256, 3, device="cuda:0", dtype=torch.int32)
        for i in range(150):
            obs, rew, reset, extras = env.step(torch.rand(256, 1, device="cuda:0", generator=g) * 2 - 1)
            if i == 60:   # a root write after the step: the pushes of the next simulate see the new pose
                r = env.root_tensor.clone()
                r[:, 3:7] = torch.tensor([0.0, 0.0, 0.2955202, 0.9553365], device="cuda:0")
                env.sim.set_actor_root_state_indexed(r, ids)
        torch.cuda.synchronize()
        out.append([t.detach().cpu().clone() for t in (obs["obs"], rew, reset, extras["time_outs"], env.root_tensor,
                                                        env.sim.dof_pos_target, env.sim.dof_vel_target,
                                                        env.progress_buf)])
        assert int(out[-1][2].sum()) >= 0
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_gpu_paper_inplace_seat_composites_equal_a_full_compose():
    """GogoroPaper resets draw new seat windows (base_x/y/z, paper.py:681-688);
    on the V12 model (codegen FUSED bit 4) the post kernel updates the rider's
    composite in place (tl_update) instead of marking the env for a compose.
    After 80 steps with many resets the composite every env holds equals a
    from-scratch compose (tg_composite) to fp32 rounding -- and the in-place
    path was taken (no env left dirty)."""
    _cuda()
    import ctypes as C
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd._lib import lib
    from thormang_isaacgym_amd.model import codegen
    n = 512
    with switches(FLIPPED):   # free base, random seat windows and steering damping
        env = tia.make(seed=21, task="GogoroPaper", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
        m = env.sim.model
        assert codegen.fused_tasks(m) & 4 and codegen.translating_locks(m, abi.ModelDesc(m).arrays)["NTL"] == 3
        g = torch.Generator(device="cuda:0").manual_seed(6)
        n_reset = 0
        for t in range(80):
            if t % 8 == 0:   # flag a random quarter of the envs: the next post-physics resets them
                env.reset_buf[torch.rand(n, device="cuda:0", generator=g) < 0.25] = 1
            n_reset += int(env.reset_buf.sum())
            env.step(torch.rand(n, 1, device="cuda:0", generator=g) * 2 - 1)
        torch.cuda.synchronize()
    assert n_reset > 20
    assert int(env.sim.env_dirty.sum()) == 0   # the resets left nothing to compose
    kc_main = 24 * m.num_groups + 12 * len(m.shapes)
    out = [torch.empty(n * 4096, device="cuda:0") for _ in range(2)]
    for k, rec in enumerate((0, 1)):
        assert lib().tg_composite(env.sim.handle, C.c_void_p(out[k].data_ptr()), rec) == 0
    torch.cuda.synchronize()
    t = codegen.translating_locks(m, abi.ModelDesc(m).arrays)
    kc = kc_main + t["KX"] + ((3 * m.num_bodies + 3) & ~3)   # + the link com block
    a = out[0][: n * kc].view(n, kc)[:, :kc_main]
    b = out[1][: n * kc].view(n, kc)[:, :kc_main]
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    err = (a - b).abs() / (1.0 + b.abs())
    assert float(err.max()) < 2e-6, float(err.max())

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


def _paper_trace(monkeypatch, env_vars, n=256, steps=150, timing_window=0):
    """Step a GogoroPaper env under the given library switches (read when the
    sim is created) with seeded random actions and a root write after step 60
    (the pushes of the next simulate see the new pose); returns its buffers
    and, with timing_window > 0, the step-kernel launches windowed timing saw
    over the last 48 steps (a window any other launch falls into is dropped)."""
    import thormang_isaacgym_amd as tia
    for k in ("TG_PAPER_UNFUSED", "TG_PAPER_TWO_LAUNCH"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env_vars.items():
        monkeypatch.setenv(k, v)
    env = tia.make(seed=11, task="GogoroPaper", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(9)
    ids = torch.arange(0, n, 3, device="cuda:0", dtype=torch.int32)
    launches = None
    for i in range(steps):
        if timing_window and i == steps - 48:
            env.sim.read_kernel_timing()
            env.sim.set_kernel_timing(-timing_window)
        obs, rew, reset, extras = env.step(torch.rand(n, 1, device="cuda:0", generator=g) * 2 - 1)
        if i == 60:
            r = env.root_tensor.clone()
            r[:, 3:7] = torch.tensor([0.0, 0.0, 0.2955202, 0.9553365], device="cuda:0")
            env.sim.set_actor_root_state_indexed(r, ids)
    torch.cuda.synchronize()
    if timing_window:
        env.sim.set_kernel_timing(0)
        launches = env.sim.read_kernel_timing()[1]
    env.sim.sync()   # (raises if a one-launch batch sum had timed out)
    out = [t.detach().cpu().clone() for t in (obs["obs"], rew, reset, extras["time_outs"], env.root_tensor,
                                              env.sim.dof_pos_target, env.sim.dof_vel_target, env.progress_buf,
                                              env.head_perturbation, env.sim.dof_state)]
    return out, launches


PAPER_FIELDS = ("obs", "rew", "reset", "time_outs", "root", "pos_target", "vel_target", "progress", "pushes", "dof")


def test_gpu_paper_two_launch_step_equals_separate_calls(monkeypatch):
    """tg_paper_step as two launches (TG_PAPER_TWO_LAUNCH=1: the pre-physics
    inside the step kernel, which also forms reward term 7's per-env
    partials, and a post launch that sums the batch itself) against the three
    separate calls (TG_PAPER_UNFUSED=1: post kernel partials, finish launch):
    the same operations in the same order, so every buffer agrees bit for bit
    -- including the head pushes, which tg_paper_step reduces inside its post
    launch, after a root write between two steps (the pre-reduced wrenches
    then give way to the next simulate's reduction)."""
    _cuda()
    a, _ = _paper_trace(monkeypatch, {"TG_PAPER_TWO_LAUNCH": "1"})
    b, _ = _paper_trace(monkeypatch, {"TG_PAPER_UNFUSED": "1"})
    assert int(a[2].sum()) >= 0
    for x, y, what in zip(a, b, PAPER_FIELDS):
        assert torch.equal(x, y), what


def test_gpu_paper_one_launch_step_matches_two_launch(monkeypatch):
    """tg_paper_step in ONE launch (the default when the batch fits one
    workgroup per CU: the post-physics as the step kernel's PaperPost
    epilogue, reward term 7's batch sum exchanged inside the launch, the
    pushes reduced to the next simulate's wrenches by the env's 16 lanes)
    against the two-launch form.  Resets, time-outs, progress and the pushes'
    timing are identical; the rest agrees to fp32 rounding (the epilogue's
    unit is the fast-math physics unit: its libm and the link kinematics of
    the push reduction round differently), far inside north_star's 1e-3.  The
    windowed kernel timing sees only step kernels in the one-launch run (any
    other launch drops its window) and none in the two-launch run."""
    _cuda()
    one, n_one = _paper_trace(monkeypatch, {}, timing_window=4)
    two, n_two = _paper_trace(monkeypatch, {"TG_PAPER_TWO_LAUNCH": "1"}, timing_window=4)
    assert n_one >= 40 and n_two == 0, (n_one, n_two)
    diffs = {}
    for x, y, what in zip(one, two, PAPER_FIELDS):
        if what in ("reset", "time_outs", "progress"):
            assert torch.equal(x, y), what
        else:
            diffs[what] = float((x.float() - y.float()).abs().max())
    print(diffs)
    assert all(d <= 1e-4 for d in diffs.values()), diffs
    assert float(one[8].abs().max()) > 0.0   # pushes happened


def test_gpu_paper_one_launch_4096_envs_reward_term7_exact(monkeypatch):
    """The bench batch (4096 envs: 256 workgroups, one per CU, every one
    waiting on every other's term-7 block sum) takes the one-launch path and
    agrees with the two-launch step as above over 60 steps."""
    _cuda()
    one, n_one = _paper_trace(monkeypatch, {}, n=4096, steps=60, timing_window=4)
    two, _ = _paper_trace(monkeypatch, {"TG_PAPER_TWO_LAUNCH": "1"}, n=4096, steps=60)
    assert n_one >= 40
    for x, y, what in zip(one, two, PAPER_FIELDS):
        if what in ("reset", "time_outs", "progress"):
            assert torch.equal(x, y), what
        else:
            assert float((x.float() - y.float()).abs().max()) <= 1e-4, what


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

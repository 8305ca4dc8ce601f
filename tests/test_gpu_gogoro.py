"""GPU parity for the Gogoro task path through the C-ABI (libtgsim.so).

* the golden fixture generated from the reference's own task module is
  replayed through the product ``Gogoro`` env (recorded physics states and
  recorded RNG draws injected) -- task kernels vs reference;
* the full env (task kernels + HIP articulation step) is run side by side
  with the CPU oracle env on identical draws -- obs / reward / reset / timeout;
* a 4096-env run (the BASELINE config) stays finite and resets/timeouts work.
"""
import os

import numpy as np
import pytest
import torch
from tests.gpu_harness import within

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def _flags(monkeypatch, f):
    """The module switches the fixture was recorded under (gogoro_new.py:25,27),
    read by Gogoro.__init__."""
    from thormang_isaacgym_amd.tasks import gogoro as gmod
    monkeypatch.setattr(gmod, "INCREMENTAL_STEER", bool(int(f["incremental_steer"])))
    monkeypatch.setattr(gmod, "DEBUG_START_SPEED", bool(int(f["debug_start_speed"])))


FIXTURES = ["gogoro_steps.npz", "gogoro_steps_flags.npz"]


@pytest.mark.parametrize("fixture", FIXTURES)
def test_gpu_task_kernels_replay_reference_steps(fixture, monkeypatch):
    _cuda()
    from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_LOWER, TG_PROP_STIFFNESS, TG_PROP_UPPER
    from thormang_isaacgym_amd.tasks.gogoro import Gogoro
    from thormang_isaacgym_amd.tasks.gogoro_draws import RecordedDraws
    from tests.golden.make_golden import gogoro_cfg

    f = np.load(os.path.join(GOLDEN, fixture))
    _flags(monkeypatch, f)
    n = int(f["n_envs"])
    src = RecordedDraws(f["draw_kind"], f["draw_size"], f["draw_vals"])
    state = {"t": 0}

    class Replay(Gogoro):
        draw_source = src
        env_spacing = 0.0

        def simulate(self):   # physics replaced by the recorded post-simulate states
            t = state["t"]
            self.root_tensor.copy_(torch.from_numpy(f["sim_root"][t]))
            self.state_dof.copy_(torch.from_numpy(f["sim_dof"][t]))
            self.frame_count += 1

    cfg = gogoro_cfg(n, int(f["max_steps"]), int(f["freq"]))
    cfg["sim"]["use_gpu_pipeline"] = True     # fixture cfg was recorded for the reference's CPU pipeline
    env = Replay(cfg, "cuda:0", "cuda:0", -1, True, False, False)
    assert src.i == int(f["init_n_draws_init"])
    np.testing.assert_allclose(env.root_tensor.cpu().numpy(), f["init_root"], atol=1e-6)
    np.testing.assert_array_equal(env.state_dof.cpu().numpy(), f["init_dof"])
    dni = env.dof_name_to_id
    st = dni["steering_joint"]
    seat = [dni["base_x"], dni["base_y"], dni["base_z"]]
    for t in range(f["actions"].shape[0]):
        state["t"] = t
        obs, rew, reset, extras = env.step(torch.from_numpy(f["actions"][t]).cuda())
        assert src.i == int(f["draw_end"][t])
        np.testing.assert_allclose(env.sim.dof_pos_target[:, st].cpu().numpy(), f["pos_target"][t][:, st], atol=1e-6)
        np.testing.assert_array_equal(env.sim.dof_vel_target.cpu().numpy(), f["vel_target"][t])
        np.testing.assert_array_equal(reset.cpu().numpy(), f["reset"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), f["progress"][t])
        np.testing.assert_array_equal(extras["time_outs"].cpu().numpy(), f["time_outs"][t])
        np.testing.assert_allclose(obs["obs"].cpu().numpy(), f["obs"][t], atol=2e-5, err_msg=f"step {t}")
        np.testing.assert_allclose(rew.cpu().numpy(), f["rew"][t], atol=2e-5)
        for k, a in (("curent_command", env.curent_command), ("action_history", env.action_history),
                     ("yaw_command", env.yaw_command), ("curent_speed", env.curent_speed),
                     ("steer_offsets", env.steer_offsets), ("imu_offsets", env.imu_offsets),
                     ("speed_offset", env.curent_speed_offset), ("buffer_obs", env.buffer_obs)):
            np.testing.assert_allclose(a.cpu().numpy(), f[k][t], atol=2e-5, err_msg=f"{k} step {t}")
        np.testing.assert_allclose(env.root_tensor.cpu().numpy(), f["root_after"][t], atol=1e-6)
        np.testing.assert_array_equal(env.state_dof.cpu().numpy(), f["dof_after"][t])
        props = env.sim.dof_props.cpu().numpy()
        np.testing.assert_allclose(props[TG_PROP_DAMPING, :, st], f["steer_damping"][t], rtol=1e-6)
        np.testing.assert_array_equal(props[TG_PROP_STIFFNESS, :, st], f["steer_stiffness"][t])
        np.testing.assert_allclose(props[TG_PROP_LOWER][:, seat], f["seat_lower"][t], atol=1e-7)
        np.testing.assert_allclose(props[TG_PROP_UPPER][:, seat], f["seat_upper"][t], atol=1e-7)
    assert src.i == len(f["draw_kind"])


@pytest.mark.parametrize("fixture", FIXTURES)
def test_gpu_fused_step_replays_reference_steps(fixture, monkeypatch):
    """The golden fixture through the TIMED path: ``Gogoro.step`` ->
    tg_gogoro_step, one launch of the step kernel with the pre-physics at its
    start and the GogoroPost epilogue (masked resets with in-place seat
    composites, observations, reward, noise, command resample), the recorded
    draws injected through its draw arrays.  The recorded post-simulate
    physics state is written into the sim before each step and the sim runs
    with 0 substeps (tg_set_sim_params), so the kernel passes it through to
    its epilogue.  Differences from the separate-call replay above, both the
    step kernel's semantics: the root state makes a frame round trip through
    the kernel (2e-6), and a locked dof of a non-reset env is stored at the
    centre of its lock window (the simulated state), not the fixture's
    synthetic value.  The second fixture flips the module's INCREMENTAL_STEER
    and DEBUG_START_SPEED switches (absolute steering, reset envs at 1.3 m/s)."""
    _cuda()
    from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_LOWER, TG_PROP_STIFFNESS, TG_PROP_UPPER
    from thormang_isaacgym_amd.tasks.gogoro import Gogoro
    from thormang_isaacgym_amd.tasks.gogoro_draws import RecordedDraws
    from tests.golden.make_golden import gogoro_cfg

    f = np.load(os.path.join(GOLDEN, fixture))
    _flags(monkeypatch, f)
    n = int(f["n_envs"])
    src = RecordedDraws(f["draw_kind"], f["draw_size"], f["draw_vals"])

    class Fused(Gogoro):
        draw_source = src
        env_spacing = 0.0

    cfg = gogoro_cfg(n, int(f["max_steps"]), int(f["freq"]))
    cfg["sim"]["use_gpu_pipeline"] = True
    env = Fused(cfg, "cuda:0", "cuda:0", -1, True, False, False)
    assert not env._replays_physics()
    sp = env.sim.get_sim_params()
    sp.substeps = 0
    env.sim.set_sim_params(sp)
    assert src.i == int(f["init_n_draws_init"])
    dni = env.dof_name_to_id
    st = dni["steering_joint"]
    seat = [dni["base_x"], dni["base_y"], dni["base_z"]]
    D = env.num_dof
    locked = np.asarray(env.sim.desc.arrays["dof_locked"], bool)
    assert locked.sum() == 34 and (~locked).sum() == 5
    n_reset = 0
    for t in range(f["actions"].shape[0]):
        env.root_tensor.copy_(torch.from_numpy(f["sim_root"][t]))
        env.state_dof.copy_(torch.from_numpy(f["sim_dof"][t]))
        was_reset = env.reset_buf.cpu().numpy().copy()   # the envs this step's epilogue resets
        obs, rew, reset, extras = env.step(torch.from_numpy(f["actions"][t]).cuda())
        assert src.i == int(f["draw_end"][t])
        np.testing.assert_allclose(env.sim.dof_pos_target[:, st].cpu().numpy(), f["pos_target"][t][:, st], atol=1e-6)
        np.testing.assert_array_equal(env.sim.dof_vel_target.cpu().numpy(), f["vel_target"][t])
        np.testing.assert_array_equal(reset.cpu().numpy(), f["reset"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), f["progress"][t])
        np.testing.assert_array_equal(extras["time_outs"].cpu().numpy(), f["time_outs"][t])
        np.testing.assert_allclose(obs["obs"].cpu().numpy(), f["obs"][t], atol=2e-5, err_msg=f"step {t}")
        np.testing.assert_allclose(rew.cpu().numpy(), f["rew"][t], atol=2e-5)
        for k, a in (("curent_command", env.curent_command), ("action_history", env.action_history),
                     ("yaw_command", env.yaw_command), ("curent_speed", env.curent_speed),
                     ("steer_offsets", env.steer_offsets), ("imu_offsets", env.imu_offsets),
                     ("speed_offset", env.curent_speed_offset), ("buffer_obs", env.buffer_obs),
                     ("config_vector", env.config_vector)):
            np.testing.assert_allclose(a.cpu().numpy(), f[k][t], atol=2e-5, err_msg=f"{k} step {t}")
        np.testing.assert_allclose(env.root_tensor.cpu().numpy(), f["root_after"][t], atol=2e-6)
        dof = env.state_dof.cpu().numpy().reshape(n, D, 2)
        ref = f["dof_after"][t].reshape(n, D, 2)
        props = env.sim.dof_props.cpu().numpy()
        r = was_reset != 0
        n_reset += int(r.sum())
        np.testing.assert_array_equal(dof[r], ref[r])                       # reset envs: the reset pose
        np.testing.assert_array_equal(dof[~r][:, ~locked], ref[~r][:, ~locked])   # active dofs pass through
        centre = 0.5 * (props[TG_PROP_LOWER] + props[TG_PROP_UPPER])
        np.testing.assert_allclose(dof[~r][:, locked, 0], centre[~r][:, locked], atol=1e-7)
        np.testing.assert_array_equal(dof[~r][:, locked, 1], 0.0)
        np.testing.assert_allclose(props[TG_PROP_DAMPING, :, st], f["steer_damping"][t], rtol=1e-6)
        np.testing.assert_array_equal(props[TG_PROP_STIFFNESS, :, st], f["steer_stiffness"][t])
        np.testing.assert_allclose(props[TG_PROP_LOWER][:, seat], f["seat_lower"][t], atol=1e-7)
        np.testing.assert_allclose(props[TG_PROP_UPPER][:, seat], f["seat_upper"][t], atol=1e-7)
    assert src.i == len(f["draw_kind"])
    assert n_reset > 0


def test_gpu_env_matches_oracle_env():
    """Task kernels + HIP articulation step vs CPU oracle env, identical draws.
    Tolerance 1e-3 on obs/reward (north_star), exact on reset/timeout."""
    _cuda()
    from tests.gpu_harness import balance_policy, gogoro_env_vs_oracle
    err = gogoro_env_vs_oracle(num_envs=128, steps=150, seed=11, policy=balance_policy)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_env_4096_runs_with_resets_and_timeouts():
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg("Gogoro", num_envs=4096)
    cfg["env"]["max_steps"] = 60
    env = tia.make(seed=42, task="Gogoro", num_envs=4096, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
    obs = env.reset()["obs"]
    assert obs.shape == (4096, 6)
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    n_reset = n_to = 0
    for _ in range(130):
        a = torch.rand(4096, 1, device="cuda:0", generator=g) * 2 - 1
        obs, rew, reset, extras = env.step(a)
        n_reset += int(reset.sum())
        n_to += int(extras["time_outs"].sum())
    assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    assert torch.isfinite(env.root_tensor).all()
    assert n_reset > 4096 and n_to > 0
    assert obs["obs"].dtype == torch.float32 and reset.dtype == torch.long and extras["time_outs"].dtype == torch.bool


def test_gpu_env_step_matches_oracle_along_1000_steps():
    """north_star horizon (1000 steps, episodes capped at 300 so every env times
    out and re-spawns): before every step the oracle env is re-synced from the
    GPU env's state (teacher forcing), so each step's obs / reward / reset /
    timeout is compared from identical inputs along the whole trajectory.  The
    free-running comparison (test_gpu_env_matches_oracle_env) covers 150 steps:
    beyond that, fp32-vs-fp64 trajectories of this balance task eventually cross
    the roll >= 0.30 termination threshold on different steps."""
    _cuda()
    from tests.gpu_harness import gogoro_forced
    err = gogoro_forced(num_envs=64, steps=1000, seed=21)
    print(err)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_4096_envs_step_matches_oracle():
    """BASELINE config 2's batch (Gogoro, 4096 envs, cfg/task/Gogoro.yaml:6)
    against the oracle env: 100 teacher-forced steps of every env under the
    bench's own action distribution (U(-1,1) steering increments: the
    scooters swerve and fall, so resets, re-spawns and the in-place seat
    composites run at the headline batch), the reference's 1000-step episode
    length."""
    _cuda()
    from tests.gpu_harness import gogoro_forced
    rs = np.random.default_rng(4096)
    err = gogoro_forced(num_envs=4096, steps=100, seed=23, max_steps=1000, threads=16,
                        policy=lambda o: rs.uniform(-1, 1, (o.shape[0], 1)).astype(np.float32))
    print(err)
    assert err["resets"] > 2048, err      # the scooters fall and re-spawn along the way
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


def test_gpu_gogoro_inplace_seat_composites_equal_a_full_compose():
    """The fused epilogue's resets move only the seat locks (base_x/y/z), so it
    updates the rider group's composite and the placements below the seat in
    place from stored mass moments (articulation_kernels.h tl_update) instead
    of re-composing the env.  After 60 steps with hundreds of such resets, the
    composite cache every env holds equals a from-scratch compose of every env
    (tg_composite instrumentation) to fp32 rounding."""
    _cuda()
    import ctypes as C
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd._lib import lib
    n = 1024
    env = tia.make(seed=33, task="Gogoro", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(4)
    n_reset = 0
    for _ in range(60):
        env.step(torch.rand(n, 1, device="cuda:0", generator=g) * 2 - 1)
        n_reset += int(env.reset_buf.sum())
    torch.cuda.synchronize()
    assert n_reset > 100
    m = env.sim.model
    kc_main = 24 * m.num_groups + 12 * len(m.shapes)      # CompLayout::ext(): the part the step kernel reads
    out = [torch.empty(n * 4096, device="cuda:0") for _ in range(2)]
    for k, rec in enumerate((0, 1)):
        assert lib().tg_composite(env.sim.handle, C.c_void_p(out[k].data_ptr()), rec) == 0
    torch.cuda.synchronize()
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.model import codegen
    kc = kc_main + codegen.translating_locks(m, abi.ModelDesc(m).arrays)["KX"]
    a = out[0][: n * kc].view(n, kc)[:, :kc_main]
    b = out[1][: n * kc].view(n, kc)[:, :kc_main]
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    err = (a - b).abs() / (1.0 + b.abs())
    assert float(err.max()) < 2e-6, float(err.max())


def test_gpu_gogoro_fused_step_matches_separate_calls():
    """tg_gogoro_step (pre-physics and post-physics in the step kernel, reset
    envs' seat composites updated in place by the epilogue) against
    tg_gogoro_pre_physics + tg_simulate + tg_gogoro_post_physics (the
    VecTask.step sequence: separate post kernel, reset envs re-composed) with
    in-kernel Philox draws, resets included.  The two paths run different
    instantiations of the fast-math step kernel and form the reset composites
    two ways (2e-6 apart, test above), and random steering amplifies that; so
    the comparison is the north_star tolerance 1e-3 over 40 free-running
    steps, while resets and progress must be identical."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.tasks.base.vec_task import VecTask
    envs = [tia.make(seed=21, task="Gogoro", num_envs=512, sim_device="cuda:0", rl_device="cuda:0")
            for _ in range(2)]
    f, u = envs
    g = torch.Generator(device="cuda:0").manual_seed(9)
    n_reset = 0
    for _ in range(40):
        a = torch.rand(512, 1, device="cuda:0", generator=g) * 2 - 1
        f.step(a)
        VecTask.step(u, a)
        torch.cuda.synchronize()
        assert torch.equal(f.reset_buf, u.reset_buf) and torch.equal(f.progress_buf, u.progress_buf)
        for x, y, what in ((f.obs_buf, u.obs_buf, "obs"), (f.rew_buf, u.rew_buf, "rew"),
                           (f.root_tensor, u.root_tensor, "root")):
            d = float((x - y).abs().max())
            assert d <= 1e-3, (what, d)
        n_reset += int(f.reset_buf.sum())
    assert n_reset > 0


def test_gpu_cpu_pipeline_config_1_delivers_the_gpu_results_on_the_host():
    """BASELINE config 1 (reference: Gogoro, 64 envs, sim_device=cpu,
    rl_device=cpu, pipeline=cpu): the env simulates on the GPU (there is no
    CPU physics outside the oracle) and hands obs / rew / reset / time_outs to
    the learner on the CPU -- the same values, bit for bit, as the GPU
    pipeline with the same seed."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    outs = []
    for sim_dev, rl_dev, gpu_pipe in (("cpu", "cpu", False), ("cuda:0", "cuda:0", True)):
        cfg = load_task_cfg("Gogoro", num_envs=64)
        cfg["sim"]["use_gpu_pipeline"] = gpu_pipe
        if not gpu_pipe:
            with pytest.warns(UserWarning, match="CPU pipeline"):
                env = tia.make(seed=7, task="Gogoro", num_envs=64, sim_device=sim_dev, rl_device=rl_dev, cfg=cfg)
        else:
            env = tia.make(seed=7, task="Gogoro", num_envs=64, sim_device=sim_dev, rl_device=rl_dev, cfg=cfg)
        g = torch.Generator().manual_seed(99)
        rec = []
        for _ in range(40):
            a = torch.rand(64, 1, generator=g) * 2 - 1
            obs, rew, reset, extras = env.step(a.to(rl_dev))
            assert obs["obs"].device == torch.device(rl_dev) and rew.device == torch.device(rl_dev)
            assert reset.device == torch.device(rl_dev) and extras["time_outs"].device == torch.device(rl_dev)
            rec.append([x.detach().cpu().clone() for x in (obs["obs"], rew, reset, extras["time_outs"])])
        outs.append(rec)
        del env
    for a, b in zip(*outs):
        for x, y in zip(a, b):
            assert torch.equal(x, y)

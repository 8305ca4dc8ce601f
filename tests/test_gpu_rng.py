"""The production random-number path on the GPU (no draw_source injected).

1. The device Philox4x32-10 (tg_rng_fill) against the Random123 known-answer
   vector and the host block function (itself KAT-pinned, tests/test_rng.py);
   its u01 / gauss transforms bit-for-bit / to the fast-math tolerance, and
   their moments.
2. Every draw kind the task kernels make, at 4096 envs, against the
   distribution the reference draws it from (tasks/gogoro_new.py:362,451-460,
   474-601; the walk task's own cfg): range, mean, variance and a
   Kolmogorov-Smirnov test.  Seeds are fixed, so every check is deterministic;
   the bounds are 6 standard errors (KS: p > 1e-6).
"""
import ctypes as C
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 4096


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def _mean_var_ok(x, mean, var, what, kurt=3.0):
    x = np.asarray(x, np.float64)
    n = x.size
    m, v = x.mean(), x.var()
    assert abs(m - mean) <= 6 * math.sqrt(var / n), (what, "mean", m, mean)
    # SE of the sample variance: var * sqrt((kurtosis - 1) / n)
    assert abs(v - var) <= 6 * var * math.sqrt((kurt - 1) / n), (what, "var", v, var)


def _ks_ok(x, cdf, what):
    from scipy import stats
    r = stats.kstest(np.asarray(x, np.float64), cdf)
    assert r.pvalue > 1e-6, (what, r)


def _uniform_ok(x, lo, hi, what):
    x = np.asarray(x, np.float64)
    assert x.min() >= lo - 1e-6 and x.max() <= hi + 1e-6, (what, x.min(), x.max())
    _mean_var_ok(x, 0.5 * (lo + hi), (hi - lo) ** 2 / 12.0, what, kurt=1.8)
    from scipy import stats
    _ks_ok(x, stats.uniform(loc=lo, scale=hi - lo).cdf, what)


def _normal_ok(x, mu, sd, what):
    _mean_var_ok(x, mu, sd * sd, what)
    from scipy import stats
    _ks_ok(x, stats.norm(loc=mu, scale=sd).cdf, what)


def _fill(kind, seed, counter, n):
    from thormang_isaacgym_amd import _lib
    from thormang_isaacgym_amd.sim import Sim, load_model
    from thormang_isaacgym_amd import abi
    sim = Sim(load_model("kat_sphere"), abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1}, {}, 1), 1, "cuda:0")
    per = 2 if kind == 2 else 4
    out = torch.zeros(n * per, dtype=torch.float32, device="cuda:0")
    _lib.check(_lib.lib().tg_rng_fill(sim.handle, kind, seed, counter, C.c_void_p(out.data_ptr()), n), "rng_fill")
    torch.cuda.synchronize()
    sim.close()
    return out.cpu()


def test_gpu_philox_words_match_kat_and_host():
    _cuda()
    from tests.test_rng import KAT, philox_np
    w = _fill(0, 0, 0, N).view(torch.int32).numpy().view(np.uint32).reshape(N, 4)
    assert tuple(int(x) for x in w[0]) == KAT[0][2]            # ctr 0, key 0
    seed, counter = 0x123456789ABCDEF0, 0x0FEDCBA987654321
    w = _fill(0, seed, counter, N).view(torch.int32).numpy().view(np.uint32).reshape(N, 4)
    i = np.arange(N, dtype=np.uint64)
    ref = philox_np((i, np.full(N, counter & 0xFFFFFFFF, np.uint64), np.full(N, counter >> 32, np.uint64),
                     np.zeros(N, np.uint64)), (np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32)))
    assert np.array_equal(w, ref)


def test_gpu_uniform_and_normal_transforms():
    _cuda()
    from tests.test_rng import philox_np
    seed, counter = 77, 5
    u = _fill(1, seed, counter, N).numpy().reshape(N, 4)
    i = np.arange(N, dtype=np.uint64)
    words = philox_np((i, np.full(N, counter, np.uint64), np.zeros(N, np.uint64), np.zeros(N, np.uint64)),
                      (np.uint64(seed), np.uint64(0)))
    want = (words >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
    assert np.array_equal(u, want)                              # u01: exact
    assert u.min() >= 0.0 and u.max() < 1.0
    _uniform_ok(u.ravel(), 0.0, 1.0, "u01")
    g = _fill(2, seed, counter, N).numpy().reshape(N, 2)
    u1 = ((words[:, [0, 2]] >> 8).astype(np.float64) + 1.0) / 16777217.0
    u2 = (words[:, [1, 3]] >> 8).astype(np.float64) / 16777216.0
    gref = np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * np.pi * u2)
    assert np.abs(g - gref).max() < 1e-4                        # __logf / __cosf fast intrinsics
    _normal_ok(g.ravel(), 0.0, 1.0, "gauss")


def test_gpu_gogoro_reset_and_noise_draws_follow_the_reference_distributions():
    """Gogoro at 4096 envs with its in-kernel draws: the initial reset_idx of
    every env (gogoro_new.py:474-601), then a step's sensor noise
    (:451-460) and pre-physics steering noise (:362)."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_LOWER, TG_PROP_UPPER
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg("Gogoro", num_envs=N)
    cfg["task"]["randomization_params"] = {"frequency": 10 ** 9}
    env = tia.make(seed=5, task="Gogoro", num_envs=N, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
    torch.cuda.synchronize()
    nz = cfg["noises"]
    dni = env.dof_name_to_id
    _uniform_ok(env.curent_speed.cpu(), *nz["speed_range"], "speed U[4,13]")
    _uniform_ok(env.curent_speed_offset.cpu(), *nz["speed_sensor_offset"], "speed offset")
    _uniform_ok(env.yaw_command.cpu(), -math.pi, math.pi, "yaw command U(-pi,pi)")
    q = env.root_tensor[:, 3:7].cpu().double()
    spawn_yaw = torch.atan2(2 * (q[:, 3] * q[:, 2] + q[:, 0] * q[:, 1]), 1 - 2 * (q[:, 1] ** 2 + q[:, 2] ** 2))
    dy = torch.remainder(spawn_yaw - env.yaw_command.cpu().double() + math.pi, 2 * math.pi) - math.pi
    _uniform_ok(dy, -1.57, 1.57, "spawn yaw - target U[-1.57,1.57]")
    props = env.sim.dof_props.cpu()
    _uniform_ok(props[TG_PROP_DAMPING][:, dni["steering_joint"]], *nz["steering_damping_range"], "steering Kd")
    for k, key in enumerate(("seat_offset_x_range", "seat_offset_y_range", "seat_offset_z_range")):
        b = dni[("base_x", "base_y", "base_z")[k]]
        lo = props[TG_PROP_LOWER][:, b]
        assert torch.allclose(props[TG_PROP_UPPER][:, b] - lo, torch.full_like(lo, 1e-4), atol=1e-6)
        _normal_ok(lo, *nz[key], key)
        _normal_ok(env.config_vector[:, k].cpu(), *nz[key], key + " (config_vector)")
    _normal_ok(env.imu_offsets.cpu(), *nz["seat_offset_xr_range"], "imu offset")
    _normal_ok(env.steer_offsets.cpu(), *nz["steering_offset"], "steer offset")
    # one step: sensor noise on the observation, steering noise on the target
    env.step(torch.zeros(N, 1, device="cuda:0"))
    torch.cuda.synchronize()
    clean = env.buffer_obs[:, -1, :].cpu().double()
    obs = env.obs_buf.cpu().double()
    live = env.progress_buf.cpu() > 0                      # envs not reset by this step
    assert int(live.sum()) > N // 2
    _normal_ok((obs[:, 0] - clean[:, 0] - env.imu_offsets.cpu().double())[live], *nz["imu_filter_noise"], "imu filter")
    _normal_ok((obs[:, 1] - clean[:, 1])[live], *nz["imu_noise"], "imu noise 1")
    _normal_ok((obs[:, 2] - clean[:, 2])[live], *nz["imu_noise"], "imu noise 2")
    assert torch.equal(obs[:, 3][live], torch.round(clean[:, 4])[live])   # the obs[3] quirk (:455-458)
    _normal_ok((obs[:, 4] - clean[:, 4])[live], *nz["imu_filter_noise"], "imu filter (delta yaw)")
    assert torch.equal(obs[:, 5], clean[:, 5])
    st = dni["steering_joint"]
    tgt = env.sim.dof_pos_target[:, st].cpu().double()
    noise = tgt - env.curent_command.cpu().double() - env.steer_offsets.cpu().double()
    _normal_ok(noise, *nz["steering_action_noise"], "steering action noise")


def test_gpu_walk_reset_and_push_draws():
    """ThormangWalkDR at 4096 envs: the constructor resets every env (commands
    U[ranges], yaw U(-pi,pi), joint positions default + U(-1,1) x jointNoise,
    joint velocities 0.1 U(-1,1)); pushes of pushForce x U(-1,1) (x, y) and
    0.25 x (z) on the push steps."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg("ThormangWalkDR", num_envs=N)
    env = tia.make(seed=11, task="ThormangWalkDR", num_envs=N, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
    torch.cuda.synchronize()   # the constructor's reset_idx of every env
    e = cfg["env"]
    r = e["randomCommandVelocityRanges"]
    cmd = env.commands.cpu()
    _uniform_ok(cmd[:, 0], *r["linear_x"], "cmd vx")
    _uniform_ok(cmd[:, 1], *r["linear_y"], "cmd vy")
    _uniform_ok(cmd[:, 2], *r["yaw"], "cmd wz")
    q = env.root_tensor[:, 3:7].cpu().double()
    assert torch.allclose(q[:, :2], torch.zeros_like(q[:, :2]))
    yaw = 2 * torch.atan2(q[:, 2], q[:, 3])
    yaw = torch.remainder(yaw + math.pi, 2 * math.pi) - math.pi
    _uniform_ok(yaw, -math.pi, math.pi, "spawn yaw")
    default = torch.as_tensor(env.default_dof_pos, dtype=torch.float64).cpu()
    jn = float(e["jointNoise"])
    dq = (env.dof_pos.cpu().double() - default) / jn
    dqd = env.dof_vel.cpu().double() / 0.1
    for d in (0, env.num_dof // 2, env.num_dof - 1):
        _uniform_ok(dq[:, d], -1.0, 1.0, f"joint noise dof {d}")
        _uniform_ok(dqd[:, d], -1.0, 1.0, f"joint velocity noise dof {d}")
    _uniform_ok(dq.ravel()[:: 7], -1.0, 1.0, "joint noise (all dofs)")
    # pushes: step until the first push step (progress % interval == 0)
    pf = float(e["learn"]["pushForce"])
    for _ in range(int(env.params.push_interval)):
        env.step(torch.zeros(N, env.num_actions, device="cuda:0"))
    torch.cuda.synchronize()
    f = env.sim.body_force.cpu().double()[:, 0, :]
    pushed = (f[:, 0] != 0) | (f[:, 1] != 0)
    assert int(pushed.sum()) > N // 2
    _uniform_ok(f[pushed, 0] / pf, -1.0, 1.0, "push x")
    _uniform_ok(f[pushed, 1] / pf, -1.0, 1.0, "push y")
    _uniform_ok(f[pushed, 2] / (0.25 * pf), -1.0, 1.0, "push z")
    assert torch.equal(f[:, 3:], torch.zeros_like(f[:, 3:]))

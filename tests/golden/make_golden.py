"""Generate the committed golden fixtures for the Gogoro task path.

RUNS ONLY IN THE BUILD CONTAINER (needs /root/reference).  It imports the
reference's own ``isaacgymenvs/tasks/gogoro_new.py`` and
``isaacgymenvs/tasks/base/vec_task.py`` behind the shim package in
``tests/golden/shim`` (our restatement of ``isaacgym.torch_utils`` plus
recorder stubs for ``gymapi``/``gymtorch``) and drives:

* ``compute_gogoro_observations``  (gogoro_new.py:692-723)      -> gogoro_obs.npz
* ``compute_gogoro_reward``        (gogoro_new.py:645-684)      -> gogoro_reward.npz
* a full ``VecTask.step`` loop      (vec_task.py:313-359 with gogoro_new.py
  pre_physics_step :347-369, post_physics_step :373-420, compute_obs_rwd
  :424-462, reset_idx :505-591) on a fake sim whose "physics" is a seeded
  synthetic random walk; every torch.rand/randn draw the reference makes is
  recorded (order, size, raw values) so the build can replay them
                                                                -> gogoro_steps.npz
* the same loop with the module's two other switches flipped:
  INCREMENTAL_STEER = False (absolute steering, gogoro_new.py:355-356) and
  DEBUG_START_SPEED = True (reset envs start at 1.3 m/s, :542-545)
                                                                -> gogoro_steps_flags.npz

Only data (inputs + outputs) is written; no reference source leaves the
container.  Re-run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/isaacgymenvs"
ASSETS = "/root/reference/assets/urdf/gogoro"


# --------------------------------------------------------------------------- import
class _Box:
    def __init__(self, *a, **k):
        pass


def load_reference():
    sys.path.insert(0, os.path.join(HERE, "shim"))
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    spaces.Box = _Box
    gym.spaces = spaces
    gym.Space = _Box
    sys.modules.setdefault("gym", gym)
    sys.modules.setdefault("gym.spaces", spaces)
    perlin = types.ModuleType("perlin_noise")
    perlin.PerlinNoise = object
    sys.modules.setdefault("perlin_noise", perlin)
    for name in ("isaacgymenvs", "isaacgymenvs.tasks", "isaacgymenvs.tasks.base", "isaacgymenvs.utils"):
        sys.modules.setdefault(name, types.ModuleType(name))
    dr = types.ModuleType("isaacgymenvs.utils.dr_utils")
    for fn in ("get_property_setter_map", "get_property_getter_map", "get_default_setter_args",
               "apply_random_samples", "check_buckets", "generate_random_samples"):
        setattr(dr, fn, lambda *a, **k: None)
    sys.modules["isaacgymenvs.utils.dr_utils"] = dr

    def _load(modname, path):
        spec = importlib.util.spec_from_file_location(modname, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
        return mod

    vt = _load("isaacgymenvs.tasks.base.vec_task", f"{REF}/tasks/base/vec_task.py")
    gg = _load("ref_gogoro_new", f"{REF}/tasks/gogoro_new.py")
    return vt, gg


# --------------------------------------------------------------------------- RNG recording
class DrawLog:
    def __init__(self):
        self.kind, self.size, self.vals = [], [], []

    def wrap(self, fn, kind):
        def f(*shape, **kw):
            t = fn(*shape, **kw)
            self.kind.append(kind)
            self.size.append(t.numel())
            self.vals.append(t.detach().reshape(-1).clone())
            return t
        return f

    def arrays(self):
        vals = torch.cat(self.vals) if self.vals else torch.zeros(0)
        return (np.array([1 if k == "n" else 0 for k in self.kind], np.int8),
                np.array(self.size, np.int64), vals.numpy().astype(np.float32))


class TorchProxy(types.ModuleType):
    def __init__(self, log):
        super().__init__("torch_proxy")
        self._log = log
        self.rand = log.wrap(torch.rand, "u")
        self.randn = log.wrap(torch.randn, "n")

    def __getattr__(self, name):
        return getattr(torch, name)


# --------------------------------------------------------------------------- fake sim
class FakeGym:
    """Records the tensor-API calls the task makes and plays a synthetic physics."""

    def __init__(self, env, num_dof, rs):
        self.env, self.D, self.rs = env, num_dof, rs
        self.pos_target = None
        self.vel_target = None
        n = env.n_envs
        self.props = {k: None for k in ("driveMode", "lower", "upper", "stiffness", "damping", "effort", "velocity")}
        self.env_props = {k: np.zeros((n, num_dof), np.float32) for k in self.props}
        self.frame = 0

    # tensor API
    def set_dof_position_target_tensor(self, sim, t):
        self.pos_target = t.clone()
        return True

    def set_dof_velocity_target_tensor(self, sim, t):
        self.vel_target = t.clone()
        return True

    def refresh_actor_root_state_tensor(self, sim):
        pass

    def refresh_dof_state_tensor(self, sim):
        pass

    def set_actor_root_state_tensor_indexed(self, sim, payload, ids, n):
        ids = ids.long()
        self.env.root_tensor[ids] = payload[ids]
        return True

    def set_dof_state_tensor_indexed(self, sim, payload, ids, n):
        return True

    def set_actor_dof_properties(self, env, handle, props):
        for k in self.env_props:
            self.env_props[k][env] = props[k]
        return True

    def clear_lines(self, v):
        pass

    def add_lines(self, *a):
        pass

    def get_frame_count(self, sim):
        return self.frame

    def fetch_results(self, sim, flag):
        pass

    def simulate(self, sim):
        """Synthetic stand-in for PhysX: a seeded random walk of the root
        attitude (some envs tip past the 0.30 rad tilt limit), random twists
        and small DOF jitter.  Only the resulting states matter: they are
        recorded and replayed verbatim by the build's parity test."""
        self.frame += 1
        rt = self.env.root_tensor
        n = rt.shape[0]
        q = rt[:, 3:7].double().numpy()
        w = self.rs.normal(0, [0.045, 0.02, 0.08], size=(n, 3))
        ang = np.linalg.norm(w, axis=1, keepdims=True)
        axis = w / np.maximum(ang, 1e-12)
        dq = np.concatenate([axis * np.sin(ang / 2), np.cos(ang / 2)], 1)
        # q <- q * dq  (xyzw)
        x1, y1, z1, w1 = q.T
        x2, y2, z2, w2 = dq.T
        qn = np.stack([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                       w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                       w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
                       w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2], 1)
        qn /= np.linalg.norm(qn, axis=1, keepdims=True)
        rt[:, 3:7] = torch.from_numpy(qn).float()
        rt[:, 7:10] = torch.from_numpy(self.rs.normal(0, 2.0, (n, 3))).float()
        rt[:, 10:13] = torch.from_numpy(self.rs.normal(0, 1.0, (n, 3))).float()
        rt[:, 0:3] += 0.03 * rt[:, 7:10]
        sd = self.env.state_dof
        sd += torch.from_numpy(self.rs.normal(0, 0.01, tuple(sd.shape))).float()


# --------------------------------------------------------------------------- env construction
def gogoro_cfg(n_envs, max_steps=1000, freq=300):
    return {
        "name": "Gogoro",
        "physics_engine": "physx",
        "env": {"numEnvs": n_envs, "max_steps": max_steps},
        "sim": {"dt": 0.03, "up_axis": "z", "use_gpu_pipeline": False, "gravity": [0.0, 0.0, -9.81], "substeps": 3},
        "noises": {
            "seat_offset_x_range": [0, 0.02], "seat_offset_y_range": [0, 0.02], "seat_offset_z_range": [0, 0.02],
            "steering_offset": [0, 0.01], "imu_filter_noise": [0, 0.001], "imu_noise": [0, 0.001],
            "seat_offset_xr_range": [0, 0.05], "speed_sensor_offset": [-0.5, 0.5], "speed_sensor_noise": [0, 0.3],
            "steering_action_noise": [0, 0.03], "spawn_x_angle": [0, 0.05], "steering_damping_range": [100, 1000],
            "IK_noise_amplitude": [0, 3], "speed_range": [4.0, 13.0],
            "speed_freq_update": freq, "yaw_freq_update": freq,
        },
        "joints_pos": {
            "l_arm_el_y": 0.0, "l_arm_wr_r": 0.0, "head_y": 0.0, "r_arm_grip": 0.0, "l_arm_wr_p": 0.0,
            "torso_y": 0.0, "r_arm_sh_r": -1.57, "l_arm_sh_p1": 0.0, "l_arm_sh_r": 1.57, "l_leg_an_r": 0.0,
            "l_leg_an_p": 0.0, "r_leg_hip_p": 1.4, "r_leg_an_p": 0.0, "l_arm_wr_y": 0.0, "l_leg_hip_p": -1.4,
            "r_leg_hip_y": 0.0, "l_leg_hip_r": 0.0, "l_leg_kn_p": 1.4, "r_arm_sh_p2": 0.0, "r_arm_sh_p1": 0.0,
            "l_leg_hip_y": 0.0, "r_leg_hip_r": 0.0, "l_arm_sh_p2": 0.0, "r_arm_wr_y": 0.0, "head_p": 0.0,
            "r_arm_wr_p": 0.0, "r_arm_wr_r": 0.0, "r_arm_el_y": 0.0, "l_arm_grip": 0.0, "r_leg_an_r": 0.0,
            "r_leg_kn_p": -1.4,
        },
        "task": {"randomize": False, "randomization_params": {"frequency": 600}},
    }


def urdf_dof_props():
    sys.path.insert(0, REPO)
    from thormang_isaacgym_amd.model.urdf import load_urdf
    m = load_urdf(f"{ASSETS}/urdf/scooter_V13.urdf", "gogoro")
    D = m.num_dof
    dt = np.dtype([("hasLimits", "?"), ("lower", "f4"), ("upper", "f4"), ("driveMode", "i4"), ("velocity", "f4"),
                   ("effort", "f4"), ("stiffness", "f4"), ("damping", "f4"), ("friction", "f4"), ("armature", "f4")])
    props = np.zeros(D, dt)
    for d, ji in enumerate(m.dof_joint):
        j = m.joints[ji]
        props["hasLimits"][d] = j.has_limits
        props["lower"][d] = j.lower if j.has_limits else -3.4e38
        props["upper"][d] = j.upper if j.has_limits else 3.4e38
        props["velocity"][d] = j.velocity
        props["effort"][d] = j.effort
    return m, props


def make_env(vt, gg, cfg, fake_rs, log):
    """Mirror of Gogoro.__init__ (gogoro_new.py:32-150) minus sim creation,
    followed by the _create_envs dof-prop setup (:246-294)."""
    G = gg.Gogoro
    g = object.__new__(G)
    model, props = urdf_dof_props()
    g.curent_step = 0
    g.device = "cpu"
    g.rl_device = "cpu"
    g.n_envs = cfg["env"]["numEnvs"]
    g.num_environments = g.n_envs
    g.max_episode_length = torch.tensor(cfg["env"]["max_steps"])
    g.randomization_params = cfg["task"]["randomization_params"]
    nz = cfg["noises"]
    g.imu_filter_noise, g.imu_noise = nz["imu_filter_noise"], nz["imu_noise"]
    g.speed_sensor_noise, g.steering_action_noise = nz["speed_sensor_noise"], nz["steering_action_noise"]
    g.spawn_x_angle, g.speed_range = nz["spawn_x_angle"], nz["speed_range"]
    g.speed_freq_update, g.yaw_freq_update = nz["speed_freq_update"], nz["yaw_freq_update"]
    g.seat_offset_x_range, g.seat_offset_y_range = nz["seat_offset_x_range"], nz["seat_offset_y_range"]
    g.seat_offset_z_range, g.seat_offset_xR_range = nz["seat_offset_z_range"], nz["seat_offset_xr_range"]
    g.steering_damping_range = nz["steering_damping_range"]
    g.steering_offset, g.speed_sensor_offset = nz["steering_offset"], nz["speed_sensor_offset"]
    n = g.n_envs
    g.imu_offsets = torch.zeros(n)
    g.steer_offsets = torch.zeros(n)
    g.curent_speed_offset = torch.zeros(n)
    g.config_vector = torch.zeros((n, 5))
    g.yaw_command = torch.zeros(n)
    g.min_speed, g.max_speed, g.max_steering, g.max_steering_change = 0.0, 10.0, 0.5, 0.2
    g.current_steering = 0.0
    g.curent_speed = g.get_randoms(n, g.speed_range)
    g.curent_command = torch.zeros(n)
    g.action_history = torch.zeros((n, 5))
    g.envs_indexes_ = torch.arange(0, n)
    g.cfg = cfg
    g.buff_size = 1
    g.buffer_obs = torch.zeros((n, 1, 6))
    g.num_observations, g.num_actions, g.num_states = 6, 1, 0
    g.control_freq_inv = 1
    g.clip_obs, g.clip_actions = math.inf, math.inf
    g.dr_randomizations = {}
    g.force_render = False
    g.extras, g.obs_dict = {}, {}
    g.sim = None
    g.viewer = None
    g.num_dof = model.num_dof
    g.dof_names = model.dof_names
    g.dof_name_to_id = {k: v for k, v in zip(g.dof_names, np.arange(g.num_dof))}
    g.num_rgbd = model.num_bodies
    g.envs = list(range(n))
    g.handles = list(range(n))
    g.gym = FakeGym(g, g.num_dof, fake_rs)
    g.apply_randomizations = lambda params: None   # dr_utils absent: DR sampling is not part of the fixture
    vt.VecTask.allocate_buffers(g)
    # _create_envs dof props (gogoro_new.py:246-294)
    g.dof_props = props
    g.thormang_pose = torch.zeros(n, g.num_dof)
    for i in range(n):
        for d in range(g.num_dof):
            g.dof_props["driveMode"][d] = 0
            g.dof_props["damping"][d] = 0.0
            g.dof_props["stiffness"][d] = 0.0
            g.dof_props["effort"][d] = 0.0
        for j_name in cfg["joints_pos"]:
            idd = g.dof_name_to_id[j_name]
            g.dof_props["lower"][idd] = cfg["joints_pos"][j_name]
            g.dof_props["upper"][idd] = g.dof_props["lower"][idd] + 0.0001
            g.thormang_pose[:, idd] = float(g.dof_props["lower"][idd] + 0.0001 / 2)
        rw, st = g.dof_name_to_id["rear_wheel_joint"], g.dof_name_to_id["steering_joint"]
        g.dof_props["driveMode"][rw] = 2
        g.dof_props["stiffness"][rw] = 0.0
        g.dof_props["damping"][rw] = 1000.0
        g.dof_props["effort"][rw] = 170.0
        g.dof_props["driveMode"][st] = 1
        g.dof_props["stiffness"][st] = 100.0
        g.dof_props["damping"][st] = 100.0
        g.dof_props["effort"][st] = 10.0
        g.dof_props["velocity"][st] = 10.0
        g.gym.set_actor_dof_properties(i, i, g.dof_props)
    # tensors (gogoro_new.py:125-145): spawn pose z=1 at env origin (0,0) here
    g.root_tensor = torch.zeros(n, 13)
    g.root_tensor[:, 2] = 1.0
    g.root_tensor[:, 6] = 1.0
    g.state_dof = torch.zeros(n * g.num_dof, 2)
    g.root_positions = g.root_tensor[:, 0:3]
    g.root_orientations = g.root_tensor[:, 3:7]
    g.root_angular_vels = g.root_tensor[:, 10:13]
    g.dof_pos = g.state_dof.view(n, g.num_dof, 2)[..., 0]
    g.dof_vel = g.state_dof.view(n, g.num_dof, 2)[..., 1]
    g.root_reset_tensor = g.root_tensor.clone().detach()
    g.root_reset_tensor[:, 7:13] = 0
    g.curent_perturbations = torch.zeros(n, g.num_rgbd, 3)
    return g, model


# --------------------------------------------------------------------------- fixtures
def random_quats(rs, n):
    u = rs.uniform(size=(n, 3))
    q = np.stack([np.sqrt(1 - u[:, 0]) * np.sin(2 * np.pi * u[:, 1]), np.sqrt(1 - u[:, 0]) * np.cos(2 * np.pi * u[:, 1]),
                  np.sqrt(u[:, 0]) * np.sin(2 * np.pi * u[:, 2]), np.sqrt(u[:, 0]) * np.cos(2 * np.pi * u[:, 2])], 1)
    return q


def euler_quat(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r / 2), np.sin(r / 2), np.cos(p / 2), np.sin(p / 2), np.cos(y / 2), np.sin(y / 2)
    return np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy], -1)


def fixture_obs(gg, rs):
    n_rand, n_up = 192, 192
    q = np.concatenate([random_quats(rs, n_rand),
                        euler_quat(rs.uniform(-0.4, 0.4, n_up), rs.uniform(-0.2, 0.2, n_up), rs.uniform(-np.pi, np.pi, n_up))])
    edge_yaw = np.array([np.pi - 1e-3, -np.pi + 1e-3, 3.0, -3.0, 0.0, 1e-4, -1e-4, np.pi / 2])
    q = np.concatenate([q, euler_quat(0.05 * np.ones(8), np.zeros(8), edge_yaw), -q[:16]])  # -q: same rotation, w<0
    n = q.shape[0]
    root = np.zeros((n, 13))
    root[:, 0:3] = rs.normal(0, 5, (n, 3))
    root[:, 3:7] = q
    root[:, 7:10] = rs.normal(0, 3, (n, 3))
    root[:, 10:13] = rs.normal(0, 2, (n, 3))
    yaw_cmd = rs.uniform(-np.pi, np.pi, n)
    yaw_cmd[:8] = [np.pi, -np.pi, np.pi - 1e-6, 0.0, 2.0, -2.0, 3.1, -3.1]
    cmd = rs.uniform(-0.5, 0.5, n)
    root32, yc32, c32 = (torch.tensor(a, dtype=torch.float32) for a in (root, yaw_cmd, cmd))
    obs = gg.compute_gogoro_observations(root32.clone(), yc32.clone(), c32.clone())
    return dict(root=root32.numpy(), yaw_command=yc32.numpy(), command=c32.numpy(), obs=obs.numpy())


def fixture_reward(gg, rs):
    n = 512
    bo = np.zeros((n, 1, 6), np.float32)
    tilt = rs.uniform(-0.5, 0.5, n)
    tilt = np.where(np.abs(np.abs(tilt) - 0.3) < 1e-3, tilt + 0.01, tilt)
    tilt[:6] = [0.0, 0.29, -0.29, 0.31, -0.31, 0.5]
    bo[:, 0, 0] = tilt
    bo[:, 0, 1] = rs.normal(0, 0.5, n)
    bo[:, 0, 2] = rs.normal(0, 1.0, n)
    bo[:, 0, 3] = rs.normal(0, 2.0, n)
    bo[:, 0, 4] = rs.uniform(-4, 4, n)
    bo[:, 0, 5] = rs.uniform(-0.5, 0.5, n)
    progress = rs.integers(0, 1002, n).astype(np.int64)
    progress[:8] = [0, 1, 997, 998, 999, 1000, 1001, 500]
    ah = rs.uniform(-1.5, 1.5, (n, 5)).astype(np.float32)
    rew, reset = gg.compute_gogoro_reward(torch.from_numpy(bo), torch.from_numpy(progress), torch.from_numpy(ah),
                                          torch.tensor(1000))
    return dict(buffer_obs=bo, progress=progress, action_history=ah, max_episode_length=np.int64(1000),
                reward=rew.numpy(), reset=reset.numpy().astype(np.int64))


def fixture_steps(vt, gg, n_envs=16, T=90, max_steps=30, freq=7, seed=1234, flags=None):
    saved = {k: getattr(gg, k) for k in (flags or {})}
    for k, v in (flags or {}).items():
        setattr(gg, k, v)
    try:
        return _fixture_steps(vt, gg, n_envs, T, max_steps, freq, seed, flags or {})
    finally:
        for k, v in saved.items():
            setattr(gg, k, v)


def _fixture_steps(vt, gg, n_envs, T, max_steps, freq, seed, flags):
    torch.manual_seed(seed)
    fake_rs = np.random.default_rng(seed + 1)
    act_rs = np.random.default_rng(seed + 2)
    log = DrawLog()
    gg.torch = TorchProxy(log)
    cfg = gogoro_cfg(n_envs, max_steps=max_steps, freq=freq)
    g, model = make_env(vt, gg, cfg, fake_rs, log)
    # reset_idx(all) at the end of __init__ (gogoro_new.py:150)
    g.reset_idx(torch.arange(0, n_envs).long())
    init = dict(root=g.root_tensor.clone().numpy(), dof=g.state_dof.clone().numpy(),
                n_draws_init=np.int64(len(log.kind)), curent_speed=g.curent_speed.clone().numpy())
    rec = {k: [] for k in ("actions", "draw_end", "sim_root", "sim_dof", "obs", "rew", "reset", "time_outs", "progress",
                           "curent_command", "action_history", "yaw_command", "curent_speed", "steer_offsets",
                           "imu_offsets", "speed_offset", "buffer_obs", "pos_target", "vel_target", "root_after",
                           "dof_after", "steer_damping", "steer_stiffness", "seat_lower", "seat_upper", "config_vector")}
    orig_sim = g.gym.simulate

    def sim_and_record(sim):
        orig_sim(sim)
        rec["sim_root"].append(g.root_tensor.clone().numpy())
        rec["sim_dof"].append(g.state_dof.clone().numpy())

    g.gym.simulate = sim_and_record
    dni = g.dof_name_to_id
    seat = [dni["base_x"], dni["base_y"], dni["base_z"]]
    st = dni["steering_joint"]
    for t in range(T):
        a = torch.from_numpy(act_rs.uniform(-1.5, 1.5, (n_envs, 1)).astype(np.float32))
        obs_dict, rew, reset, extras = vt.VecTask.step(g, a)
        rec["actions"].append(a.numpy())
        rec["draw_end"].append(len(log.kind))
        rec["obs"].append(obs_dict["obs"].clone().numpy())
        rec["rew"].append(rew.clone().numpy())
        rec["reset"].append(reset.clone().numpy())
        rec["time_outs"].append(extras["time_outs"].clone().numpy())
        rec["progress"].append(g.progress_buf.clone().numpy())
        rec["curent_command"].append(g.curent_command.clone().numpy())
        rec["action_history"].append(g.action_history.clone().numpy())
        rec["yaw_command"].append(g.yaw_command.clone().numpy())
        rec["curent_speed"].append(g.curent_speed.clone().numpy())
        rec["steer_offsets"].append(g.steer_offsets.clone().numpy())
        rec["imu_offsets"].append(g.imu_offsets.clone().numpy())
        rec["speed_offset"].append(g.curent_speed_offset.clone().numpy())
        rec["buffer_obs"].append(g.buffer_obs.clone().numpy())
        rec["pos_target"].append(g.gym.pos_target.numpy())
        rec["vel_target"].append(g.gym.vel_target.numpy())
        rec["root_after"].append(g.root_tensor.clone().numpy())
        rec["dof_after"].append(g.state_dof.clone().numpy())
        ep = g.gym.env_props
        rec["steer_damping"].append(ep["damping"][:, st].copy())
        rec["steer_stiffness"].append(ep["stiffness"][:, st].copy())
        rec["seat_lower"].append(ep["lower"][:, seat].copy())
        rec["seat_upper"].append(ep["upper"][:, seat].copy())
        rec["config_vector"].append(g.config_vector.clone().numpy())
    kinds, sizes, vals = log.arrays()
    out = {k: np.stack(v) for k, v in rec.items()}
    out.update({f"init_{k}": v for k, v in init.items()})
    out.update(draw_kind=kinds, draw_size=sizes, draw_vals=vals, n_envs=np.int64(n_envs), max_steps=np.int64(max_steps),
               freq=np.int64(freq), dof_names=np.array(model.dof_names),
               incremental_steer=np.int64(gg.INCREMENTAL_STEER), debug_start_speed=np.int64(gg.DEBUG_START_SPEED))
    return out


def main():
    vt, gg = load_reference()
    rs = np.random.default_rng(7)
    np.savez_compressed(os.path.join(HERE, "gogoro_obs.npz"), **fixture_obs(gg, rs))
    np.savez_compressed(os.path.join(HERE, "gogoro_reward.npz"), **fixture_reward(gg, rs))
    np.savez_compressed(os.path.join(HERE, "gogoro_steps.npz"), **fixture_steps(vt, gg))
    np.savez_compressed(os.path.join(HERE, "gogoro_steps_flags.npz"),
                        **fixture_steps(vt, gg, seed=4321, flags=dict(INCREMENTAL_STEER=False, DEBUG_START_SPEED=True)))
    for f in ("gogoro_obs.npz", "gogoro_reward.npz", "gogoro_steps.npz", "gogoro_steps_flags.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()

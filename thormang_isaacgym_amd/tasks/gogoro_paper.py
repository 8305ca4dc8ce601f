"""Gogoro "paper" variant (registered here as "GogoroPaper").

Drop-in mirror of the reference's unregistered
``isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py`` (class ``Gogoro``,
cfg/task/Gogoro_paper.yaml): 8 observations x 20-step history (160), a 5-slot
command history with the steering delay, noisy observation history, head
pushes and its reward.  The module-level switches keep the reference's
committed values (DEBUG = True) and are read when an env is constructed, so a
caller can flip them the way the reference's module constants are edited.

  pre_physics_step  (paper.py:349-393)             -> tg_paper_pre_physics
  gym.simulate      (vec_task.py:332-335)           -> tg_simulate
  post_physics_step (paper.py:397-482, compute_obs_rwd :491-547, reset_idx
                     :609-692, VecTask.step tail)   -> tg_paper_post_physics

Differences from the reference, all deliberate:
* resets are masked inside the post kernel (no host loop, no
  ``set_actor_dof_properties`` calls);
* the reference raises IndexError in ``speed_command_change[speed_command_change]``
  (:405-408) unless the envs due for a change are exactly {0..k-1}, and in the
  push update (:443-451) for more than 2048 envs; here the first is the identity
  (its value on every input the reference accepts) and pushes apply to the first
  ``push_max_envs`` (2048) envs at any batch size;
* draws come from an in-kernel Philox stream unless a ``draw_source``
  (tasks/paper_draws.py) replays the reference's torch.rand order;
* the viewer debug lines (:416-482) are not drawn;
* DEBUGUSETERRAIN (Perlin trimesh) is SURVEY §8 f3 and raises here.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from .. import abi
from .._lib import check, lib
from ..abi import (TG_PROP_ARMATURE, TG_PROP_DAMPING, TG_PROP_DRIVE_MODE, TG_PROP_EFFORT, TG_PROP_LOWER,
                   TG_PROP_STIFFNESS, TG_PROP_UPPER, TG_PROP_VELOCITY, default_dof_props)
from ..sim import load_model
from .base.vec_task import VecTask, pipeline_device
from .gogoro_cfg import check_lock_set, lock_window
from .paper_draws import ctor_draws, post_draws, reset_draws

# module switches of the reference (paper.py:23-34), committed values
DEBUG = True
DEBUGFIXBASE = True
DEBUGUSETERRAIN = False
DEBUG_START_SPEED = True
RANDOM_DAMPING = False
PUSH_ROBOT = DEBUG
CENTER_ROBOT = DEBUG
USE_STEER_DELAY = not DEBUG
IGNORE_ZERO = not DEBUG

#: AssetOptions of paper.py:205-212 (linear damping commented out there, default
#: armature) + plane friction :188-190; IsaacGym default angular damping 0.5
ASSET_OPTIONS = {"linear_damping": 0.0, "angular_damping": 0.5, "armature": 0.0, "ground_friction": 0.99}

HIST, NOBS, CMD_HIST = 20, 8, 5


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def paper_dof_props(model, cfg: dict, num_envs: int) -> np.ndarray:
    """[TG_NUM_PROPS, N, D] as _create_envs sets them (paper.py:250-300)."""
    dni = model.dof_name_to_id()
    props = default_dof_props(model, num_envs)
    props[TG_PROP_DRIVE_MODE] = 0
    props[TG_PROP_DAMPING] = 0
    props[TG_PROP_STIFFNESS] = 0
    props[TG_PROP_EFFORT] = 0
    lock_window(cfg, dni, props[TG_PROP_LOWER], props[TG_PROP_UPPER])
    for b in ("base_x", "base_y", "base_z"):          # :268-276 seats locked at 0
        props[TG_PROP_LOWER, :, dni[b]] = 0.0
        props[TG_PROP_UPPER, :, dni[b]] = np.float32(0.0) + np.float32(0.0001)
    rw, st = dni["rear_wheel_joint"], dni["steering_joint"]
    props[TG_PROP_DRIVE_MODE, :, rw] = 2
    props[TG_PROP_DAMPING, :, rw] = 1000.0
    props[TG_PROP_EFFORT, :, rw] = 170.0
    props[TG_PROP_DRIVE_MODE, :, st] = 1
    props[TG_PROP_STIFFNESS, :, st] = 100.0
    props[TG_PROP_DAMPING, :, st] = 100.0
    props[TG_PROP_EFFORT, :, st] = 10.0
    props[TG_PROP_VELOCITY, :, st] = 50.0
    props[TG_PROP_ARMATURE] = ASSET_OPTIONS["armature"]
    return props


def paper_pose(cfg: dict, dni: dict, num_envs: int) -> np.ndarray:
    """thormang_pose [N, D]: lock-window centres (paper.py:265,278-280)."""
    pose = np.zeros((num_envs, len(dni)), np.float32)
    for name, val in cfg["joints_pos"].items():
        pose[:, dni[name]] = np.float32(val) + np.float32(0.0001 / 2)
    for b in ("base_x", "base_y", "base_z"):
        pose[:, dni[b]] = np.float32(0.0) + np.float32(0.0001 / 2)
    return pose


def head_geometry(model, cfg: dict):
    """head_p_link COM and the root group's COM in the root frame at the lock pose."""
    dni = model.dof_name_to_id()
    q = {n: float(v) + 0.0001 / 2 for n, v in cfg["joints_pos"].items()}
    q.update({b: 0.0001 / 2 for b in ("base_x", "base_y", "base_z")})
    fk = model.forward_kinematics(q)
    h = model.link_index("head_p_link")
    R, p = fk[h]
    head = p + R @ np.asarray(model.links[h].com)
    m_tot, c = 0.0, np.zeros(3)
    for li, link in enumerate(model.links):
        if model.link_group[li] == 0:
            R, p = fk[li]
            c += link.mass * (p + R @ np.asarray(link.com))
            m_tot += link.mass
    del dni
    return head.astype(np.float32), (c / m_tot).astype(np.float32)


def paper_params(cfg: dict, model, num_envs: int, switches: dict, seed: int = 0) -> abi.tg_paper_params:
    nz = cfg["noises"]
    dni = model.dof_name_to_id()
    p = abi.tg_paper_params()
    p.num_envs, p.num_dof, p.num_groups = int(num_envs), model.num_dof, model.num_groups
    p.dof_steer, p.dof_rear = int(dni["steering_joint"]), int(dni["rear_wheel_joint"])
    p.dof_base_x, p.dof_base_y, p.dof_base_z = (int(dni[b]) for b in ("base_x", "base_y", "base_z"))
    p.max_episode_length = int(cfg["env"]["max_steps"])
    p.speed_freq_update, p.yaw_freq_update = int(nz["speed_freq_update"]), int(nz["yaw_freq_update"])
    for k in ("command_delay", "imu_filter_noise", "imu_noise", "speed_sensor_noise", "speed_sensor_offset",
              "imu_x_offset", "speed_range", "steering_offset", "steering_damping_range", "seat_offset_x_range",
              "seat_offset_y_range", "seat_offset_z_range"):
        getattr(p, k)[:] = [float(x) for x in nz[k]]
    p.max_steering, p.max_tilt, p.spawn_z, p.start_speed = 0.5, 0.38, 0.03, 1.3
    p.push_force, p.push_interval, p.push_max_envs = 30.0, 10, 2048
    p.use_steer_delay = int(bool(switches["USE_STEER_DELAY"]))
    p.random_damping = int(bool(switches["RANDOM_DAMPING"]))
    p.center_robot = int(bool(switches["CENTER_ROBOT"]))
    p.push_robot = int(bool(switches["PUSH_ROBOT"]))
    p.debug_start_speed = int(bool(switches["DEBUG_START_SPEED"]))
    p.damping_stiffness, p.damping_effort, p.damping_velocity = 13700.0, 200.0, 1.0
    head, g0 = head_geometry(model, cfg)
    p.head_com[:] = head.tolist()
    p.group0_com[:] = g0.tolist()
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return p


def current_switches() -> dict:
    g = globals()
    return {k: g[k] for k in ("DEBUGFIXBASE", "DEBUGUSETERRAIN", "DEBUG_START_SPEED", "RANDOM_DAMPING", "PUSH_ROBOT",
                              "CENTER_ROBOT", "USE_STEER_DELAY")}


class Gogoro(VecTask):
    #: optional DrawSource replaying the reference's torch.rand order (tasks/paper_draws.py)
    draw_source = None
    env_spacing = 1.0

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture, force_render):
        self.switches = current_switches()
        if self.switches["DEBUGUSETERRAIN"]:
            raise NotImplementedError("terrain (paper.py:171-187) is SURVEY §8 f3, not part of this build")
        self.steering_sensitivity = 0.1
        self.curent_step = 0
        self.device = pipeline_device(cfg, sim_device)   # the sim GPU (also for the CPU pipeline)
        self.n_envs = n = cfg["env"]["numEnvs"]
        self.max_episode_length = torch.tensor(cfg["env"]["max_steps"])
        nz = cfg["noises"]
        for k in ("imu_filter_noise", "imu_noise", "speed_sensor_noise", "speed_sensor_offset",
                  "seat_offset_x_range", "seat_offset_y_range", "seat_offset_z_range", "spawn_x_angle",
                  "imu_x_offset", "steering_damping_range", "steering_action_noise", "speed_range",
                  "speed_freq_update", "yaw_freq_update", "steering_offset", "command_delay"):
            setattr(self, k, nz[k])
        self.dof_props = None
        dev = self.device
        self.yaw_command = torch.zeros(n, device=dev)
        self.min_speed, self.max_speed, self.max_steering = 0.0, 10.0, 0.5
        self.draw_source = getattr(self, "draw_source", None)
        self._rng_counter = 1
        self.seed = int(cfg.get("seed", 42)) if isinstance(cfg.get("seed", 42), (int, float)) else 42
        # constructor draws in the reference's order (:75-90)
        if self.draw_source is not None:
            u = torch.from_numpy(ctor_draws(self.draw_source, n)).to(dev)
        else:
            u = torch.rand((n, 6), device=dev)

        def aff(col, b):
            return b[0] + u[:, col] * (b[1] - b[0])
        self.curent_speed = aff(0, self.speed_range).contiguous()
        self.last_err = torch.zeros(n, device=dev)
        self.curent_command = torch.zeros(n, device=dev)
        self.steer_offsets = aff(1, self.steering_offset).contiguous()
        self.steer_delay = aff(2, self.command_delay).to(torch.long).contiguous()
        self.command_history = torch.zeros((n, self.command_delay[1]), device=dev)
        if self.command_history.shape[1] != CMD_HIST:
            raise ValueError(f"noises.command_delay[1] must be {CMD_HIST} (the fused kernels' history width)")
        self.envs_indexes_ = torch.arange(0, n)
        self.curent_damping_cfg = aff(3, self.steering_damping_range).contiguous()
        self.curent_speed_offset = aff(4, self.speed_sensor_offset).contiguous()
        self.curent_imu_x_offset = aff(5, self.imu_x_offset).contiguous()
        self.speed_no_noise = torch.zeros(n, device=dev)
        self.integral_error = torch.zeros(n, device=dev)
        self.last_err_speed = torch.zeros(n, device=dev)
        self.viewer = virtual_screen_capture
        self.cfg = cfg
        self.buff_size = HIST
        self.buffer_obs = torch.zeros((n, HIST, NOBS), device=dev)
        self.buffer_obs_noisy = torch.zeros((n, HIST, NOBS), device=dev)
        self.cfg["env"]["numObservations"] = NOBS * HIST
        self.cfg["env"]["numActions"] = 1
        super().__init__(config=self.cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        self.dt = self.sim_params["dt"]
        self.root_tensor = self.sim.root_state
        self.state_dof = self.sim.dof_state
        self.root_positions = self.root_tensor[:, 0:3]
        self.root_orientations = self.root_tensor[:, 3:7]
        self.root_angular_vels = self.root_tensor[:, 10:13]
        self.dof_pos = self.state_dof.view(n, self.num_dof, 2)[..., 0]
        self.dof_vel = self.state_dof.view(n, self.num_dof, 2)[..., 1]
        self.root_tensor[:, 2] = 1.0                               # start pose z = 1 (paper.py:288)
        self.root_tensor[:, 6] = 1.0
        self.root_reset_tensor = self.root_tensor.clone().detach()
        self.root_reset_tensor[:, 7:13] = 0
        # the reference's [N, L, 3] perturbation tensor (:457); the post kernel
        # writes head_p_link's rows in place (tg_paper_params.perturbation_stride)
        self._perturbations = torch.zeros((n, self.num_rgbd, 3), device=dev)
        self._head_id = self.rgid_body_to_id["head_p_link"]
        self.head_perturbation = self._perturbations[:, self._head_id]   # strided view
        self.scratch = torch.zeros(n, device=dev)
        self.current_steering = None
        self.params = paper_params(self.cfg, self.model, n, self.switches, self.seed)
        self.params.perturbation_stride = 3 * self.num_rgbd
        self._bufs = self._make_buffers()
        self.reset_idx(torch.arange(0, n, device=self.device).type(torch.long))

    @property
    def curent_perturbations(self) -> torch.Tensor:
        """[N, num_rgbd, 3] the reference's perturbation tensor (:457); only head_p_link is ever pushed."""
        return self._perturbations

    # ------------------------------------------------------------ creation
    def create_sim(self):
        self.model = model = load_model("gogoro_v12")
        check_lock_set(self.cfg, model)
        asset_options = dict(ASSET_OPTIONS, fix_base_link=bool(self.switches["DEBUGFIXBASE"]))
        self.sim = self.create_sim_object(model, asset_options, env_spacing=self.env_spacing)
        self._create_envs(model)

    def _create_envs(self, model):
        self.num_dof = model.num_dof
        self.dof_names = list(model.dof_names)
        self.dof_name_to_id = {k: v for k, v in zip(self.dof_names, np.arange(self.num_dof))}
        self.num_rgbd = model.num_bodies
        self.rgid_body_to_id = {l.name: i for i, l in enumerate(model.links)}
        self.sim.dof_props.copy_(torch.from_numpy(paper_dof_props(model, self.cfg, self.n_envs)))
        self.sim.env_dirty.fill_(1)
        self.dof_props = self.sim.dof_props
        self.thormang_pose = torch.from_numpy(paper_pose(self.cfg, self.dof_name_to_id, self.n_envs)).to(self.device)

    def _make_buffers(self) -> abi.tg_paper_buffers:
        b = abi.tg_paper_buffers()
        push = bool(self.switches["PUSH_ROBOT"])
        pairs = dict(obs_buf=self.obs_buf, buffer_obs=self.buffer_obs, buffer_obs_noisy=self.buffer_obs_noisy,
                     rew_buf=self.rew_buf, reset_buf=self.reset_buf, progress_buf=self.progress_buf,
                     timeout_buf=self.timeout_buf, curent_command=self.curent_command,
                     command_history=self.command_history, steer_delay=self.steer_delay,
                     steer_offsets=self.steer_offsets, curent_speed=self.curent_speed,
                     curent_speed_offset=self.curent_speed_offset, curent_imu_x_offset=self.curent_imu_x_offset,
                     curent_damping_cfg=self.curent_damping_cfg, yaw_command=self.yaw_command,
                     speed_no_noise=self.speed_no_noise, perturbation=self.head_perturbation,
                     root_reset=self.root_reset_tensor, thormang_pose=self.thormang_pose, root=self.sim.root_state,
                     dof_state=self.sim.dof_state, pos_target=self.sim.dof_pos_target,
                     vel_target=self.sim.dof_vel_target, dof_props=self.sim.dof_props,
                     body_force=None, env_dirty=self.sim.env_dirty,
                     scratch=self.scratch)
        for k, t in pairs.items():
            if t is None:
                continue
            if k == "perturbation":   # head_p_link's rows of the [N, L, 3] tensor, stride L*3
                setattr(b, k, t.data_ptr())
                continue
            if not t.is_contiguous() or t.device != torch.device(self.device):
                raise RuntimeError(f"task buffer {k} must be contiguous on {self.device}")
            setattr(b, k, t.data_ptr())
        if self.obs_buf.shape[1] != NOBS * HIST:
            raise RuntimeError("obs_buf must be [N, 160]")
        if push:   # tg_paper_step applies the [N*L, 3] tensor to the next simulate itself (:457)
            b.rb_forces = self._perturbations.data_ptr()
        self._buf_tensors = pairs
        return b

    def _counter(self) -> int:
        self._rng_counter += 1
        return self._rng_counter

    def _dev(self, a):
        return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------ hot path
    def pre_physics_step(self, actions):
        a = actions.to(device=self.device, dtype=torch.float32).contiguous()
        check(lib().tg_paper_pre_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a),
                                         self._counter()), "tg_paper_pre_physics")
        self._keep = a

    def post_physics_step(self):
        keep = None
        if self.draw_source is not None:
            ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1).cpu().numpy()
            keep = [self._dev(x) for x in post_draws(
                self.draw_source, ids, self.progress_buf.cpu().numpy(), int(self.params.speed_freq_update),
                bool(self.params.push_robot), bool(self.params.random_damping), bool(self.params.center_robot))]
        rd, nd, sd, yd, pd = keep if keep is not None else (None,) * 5
        check(lib().tg_paper_post_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(rd), _p(nd),
                                          _p(sd), _p(yd), _p(pd), self._counter()), "tg_paper_post_physics")
        self._keep_post = keep
        self._post_host()

    def _post_host(self, applied: bool = False):
        self.curent_step += 1
        if self.switches["PUSH_ROBOT"] and not applied:   # :449-457, the reference's own [N*L, 3] tensor
            self.sim.apply_rigid_body_force_tensors(torch.flatten(self._perturbations, end_dim=-2), None)

    def compute_obs_rwd(self):
        raise NotImplementedError("compute_obs_rwd runs inside the fused post-physics kernel")

    def step(self, actions):
        if self.draw_source is None and os.environ.get("TG_PAPER_UNFUSED", "0") != "1":
            # pre_physics_step + control_freq_inv x simulate + post_physics_step in
            # one library call (tg_paper_step: the pre-physics rides in the first
            # simulate's compose launch); the same Philox counters as the separate calls
            a = actions.to(device=self.device, dtype=torch.float32).contiguous()
            self._counter()   # the pre-physics call's counter (its kernel draws nothing)
            check(lib().tg_paper_step(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a),
                                      self.control_freq_inv, self._counter()), "tg_paper_step")
            self._keep = a
            self.frame_count += self.control_freq_inv
            # (tg_paper_step applied rb_forces = the perturbation tensor already,
            # as apply_rigid_body_force_tensors right after it would)
            self._post_host(applied=bool(self._bufs.rb_forces))
        else:
            self.pre_physics_step(actions)
            for _ in range(self.control_freq_inv):
                self.simulate()
            self.post_physics_step()
        self.extras["time_outs"] = self.timeout_buf
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs) \
            if math.isfinite(self.clip_obs) else self.obs_buf
        return self._rl_out()

    # ------------------------------------------------------------ resets / draws
    def get_randoms(self, shape, bounds):
        u = self._dev(self.draw_source.uniform(int(np.prod(shape))).reshape(shape)) \
            if self.draw_source is not None else torch.rand(shape, device=self.device)
        return bounds[0] + u * (bounds[1] - bounds[0])

    def reset_idx(self, env_ids):
        env_ids = torch.as_tensor(env_ids, device=self.device)
        n = int(env_ids.numel())
        if n == 0:
            return
        ids32 = env_ids.to(torch.int32).contiguous()
        rd = None
        if self.draw_source is not None:
            rd = self._dev(reset_draws(self.draw_source, np.sort(env_ids.cpu().numpy()), self.n_envs,
                                       bool(self.params.random_damping), bool(self.params.center_robot)))
        check(lib().tg_paper_reset_idx(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(ids32), n,
                                       _p(rd), self._counter()), "tg_paper_reset_idx")
        self._keep_reset = (ids32, rd)

"""Gogoro scooter balance task (registered as "Gogoro").

Drop-in mirror of the reference's ``isaacgymenvs/tasks/gogoro_new.py``:
same class name, constructor signature, cfg schema (cfg/task/Gogoro.yaml),
attribute names, observation/action layout ([N,6] / [N,1]) and step
semantics.  ``step`` is one library call, ``tg_gogoro_step``: one launch of
the articulation step kernel with the pre-physics at its start and the
post-physics as its epilogue (libtgsim.so).  The separate-call API the
reference's method names map to stays available:

  pre_physics_step  (gogoro_new.py:347-369)  -> tg_gogoro_pre_physics
  gym.simulate      (vec_task.py:332-335)     -> tg_simulate
  post_physics_step (gogoro_new.py:373-462 incl. reset_idx :505-591 and the
                     VecTask.step tail vec_task.py:345-353) -> tg_gogoro_post_physics

Differences from the reference, all deliberate:
* resets are masked inside the post kernel (no ``reset_buf.nonzero()``, no
  per-env Python loop, no ``set_actor_dof_properties`` host calls);
* random draws come from an in-kernel Philox stream; attaching a
  ``draw_source`` (tasks/gogoro_draws.py) replays the reference's
  ``torch.rand/randn`` call order exactly (parity tests);
* the debug-line block (:392-420) -- viewer only, no buffer effects -- is not
  reproduced, which removes its ~16 device->host syncs per step;
* ``USE_TERAIN`` (:26, :157-181, :523-534) hands the Perlin height samples to
  the simulator (tg_set_heightfield) instead of a triangle mesh: the contact
  kernel evaluates that mesh's surface directly (tasks/terrain.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import abi
from .._lib import check, lib
from ..sim import load_model
from .base.vec_task import VecTask, pipeline_device
from .gogoro_cfg import ASSET_OPTIONS, check_lock_set, gogoro_params, initial_dof_props, thormang_pose
from .gogoro_draws import post_draws, reset_draws
from .terrain import Terrain

# module-level switches of the reference (gogoro_new.py:22-27), read when an
# env is created: DEBUG_START_SPEED (:25, :542-545) starts a reset env at
# 1.3 m/s along its spawn heading; INCREMENTAL_STEER = False (:27, :355-356)
# makes the command action * max_steering instead of an increment
DEBUGFIXBASE = False
DEBUG_START_SPEED = False
USE_TERAIN = False
INCREMENTAL_STEER = True


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class Gogoro(VecTask):
    #: optional DrawSource (tasks/gogoro_draws.py) replaying the reference's RNG stream
    draw_source = None

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture, force_render):
        self.curent_step = 0
        self.device = pipeline_device(cfg, sim_device)   # the sim GPU (also for the CPU pipeline)
        self.n_envs = cfg["env"]["numEnvs"]
        self.max_episode_length = torch.tensor(cfg["env"]["max_steps"])
        self.randomization_params = cfg["task"]["randomization_params"]
        nz = cfg["noises"]
        self.imu_filter_noise = nz["imu_filter_noise"]
        self.imu_noise = nz["imu_noise"]
        self.speed_sensor_noise = nz["speed_sensor_noise"]
        self.steering_action_noise = nz["steering_action_noise"]
        self.spawn_x_angle = nz["spawn_x_angle"]
        self.speed_range = nz["speed_range"]
        self.speed_freq_update = nz["speed_freq_update"]
        self.yaw_freq_update = nz["yaw_freq_update"]
        self.dof_props = None
        self.seat_offset_x_range = nz["seat_offset_x_range"]
        self.seat_offset_y_range = nz["seat_offset_y_range"]
        self.seat_offset_z_range = nz["seat_offset_z_range"]
        self.seat_offset_xR_range = nz["seat_offset_xr_range"]
        self.steering_damping_range = nz["steering_damping_range"]
        self.steering_offset = nz["steering_offset"]
        self.speed_sensor_offset = nz["speed_sensor_offset"]
        n = self.n_envs
        dev = self.device
        self.imu_offsets = torch.zeros(n, device=dev)
        self.steer_offsets = torch.zeros(n, device=dev)
        self.curent_speed_offset = torch.zeros(n, device=dev)
        self.config_vector = torch.zeros((n, 5), device=dev)
        self.yaw_command = torch.zeros(n, device=dev)
        self.min_speed, self.max_speed = 0.0, 10.0
        self.max_steering, self.max_steering_change = 0.5, 0.2
        self.current_steering = 0.0
        self.draw_source = getattr(self, "draw_source", None)
        self._rng_counter = 1
        self.seed = int(cfg.get("seed", 42)) if isinstance(cfg.get("seed", 42), (int, float)) else 42
        self.curent_speed = self.get_randoms(n, self.speed_range)
        self.curent_command = torch.zeros(n, device=dev)
        self.action_history = torch.zeros((n, 5), device=dev)
        self.envs_indexes_ = torch.arange(0, n)
        self.viewer = virtual_screen_capture
        self.cfg = cfg
        num_obs, num_acts = 6, 1
        self.buff_size = 1
        self.buffer_obs = torch.zeros((n, self.buff_size, num_obs), device=dev)
        self.cfg["env"]["numObservations"] = num_obs * self.buff_size
        self.cfg["env"]["numActions"] = num_acts
        super().__init__(config=self.cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        self.dt = self.sim_params["dt"]
        self.root_tensor = self.sim.root_state
        self.state_dof = self.sim.dof_state
        self.root_positions = self.root_tensor[:, 0:3]
        self.root_orientations = self.root_tensor[:, 3:7]
        self.root_angular_vels = self.root_tensor[:, 10:13]
        self.dof_pos = self.state_dof.view(self.n_envs, self.num_dof, 2)[..., 0]
        self.dof_vel = self.state_dof.view(self.n_envs, self.num_dof, 2)[..., 1]
        self.root_tensor[:, 2] = 1.0                               # start pose z = 1 (gogoro_new.py:280-281)
        self.root_reset_tensor = self.root_tensor.clone().detach()
        self.root_reset_tensor[:, 7:13] = 0
        self.curent_perturbations = torch.zeros(self.n_envs, self.num_rgbd, 3, device=self.device)
        self.params = gogoro_params(self.cfg, self.dof_name_to_id, self.n_envs, self.seed)
        self.params.absolute_steer = int(not INCREMENTAL_STEER)
        self.params.debug_start_speed = int(bool(DEBUG_START_SPEED))
        if self.terrain is not None:
            self.root_reset_tensor[:, 2] = self._terrain_spawn_z()
            self.params.terrain_spawn = 1
        self._bufs = self._make_buffers()
        self.reset_idx(torch.arange(0, self.n_envs, device=self.device).type(torch.long))

    # ------------------------------------------------------------ creation
    #: create_env spacing (gogoro_new.py:239); env origins form a 2*spacing grid
    env_spacing = 1.0

    def create_sim(self):
        model = load_model("gogoro")
        check_lock_set(self.cfg, model)
        asset_options = dict(ASSET_OPTIONS, fix_base_link=DEBUGFIXBASE)
        self.sim = self.create_sim_object(model, asset_options, env_spacing=self.env_spacing)
        self.terrain = None
        if USE_TERAIN:
            self._create_ground_plane()
        self._create_envs(model)
        self.apply_randomizations(self.randomization_params)

    #: grid pitch the terrain placement assumes (gogoro_new.py:171, = 2 x env_spacing)
    terrain_env_pitch = 2

    def _create_ground_plane(self):
        """The Perlin terrain beside the z = 0 plane (gogoro_new.py:164-181):
        a 512 x 512 heightfield drawn from the CPU torch generator, shifted by
        -start_mid in x and y so the env grid sits in its middle, friction 0.98."""
        self.terrain = Terrain()
        envs_scale = self.terrain_env_pitch * int(np.sqrt(self.n_envs))
        self._terrain_start_mid = int(self.terrain.Vx_size_m / 2 - envs_scale / 2)
        o = -float(self._terrain_start_mid)
        self.sim.set_heightfield(self.terrain.heightsamples, self.terrain.V_scale, self.terrain.H_scale, o, o,
                                 friction=0.98)
        self.terrain.heightsamples = self.terrain.heightsamples.to(self.device)

    def _terrain_spawn_z(self) -> torch.Tensor:
        """Per-env reset height on the terrain (gogoro_new.py:523-534): the
        height sample under the env origin, minus 0.03, clamped to [0, 100]."""
        t = self.terrain
        sq = int(np.sqrt(self.n_envs))
        smi = int(self._terrain_start_mid * (1 / t.V_scale))
        e = torch.arange(self.n_envs, device=self.device, dtype=torch.int32)
        step = self.terrain_env_pitch / t.V_scale
        ix = smi + ((e % sq) * step).to(torch.int)
        iy = smi + ((e // sq) * step).to(torch.int)
        z = t.heightsamples[ix.long(), iy.long()] * t.H_scale - 0.03
        return torch.clamp(z, 0, 100.0)

    def _create_envs(self, model):
        """DOF properties exactly as gogoro_new.py:231-294 sets them, for all envs at once."""
        self.num_dof = model.num_dof
        self.dof_names = list(model.dof_names)
        self.dof_name_to_id = {k: v for k, v in zip(self.dof_names, np.arange(self.num_dof))}
        self.num_rgbd = model.num_bodies
        self.rgid_body_to_id = {l.name: i for i, l in enumerate(model.links)}
        self.rgid_body_to_name = {i: l.name for i, l in enumerate(model.links)}
        props = initial_dof_props(model, self.cfg, self.n_envs)
        self.sim.dof_props.copy_(torch.from_numpy(props))
        self.sim.env_dirty.fill_(1)
        self.dof_props = self.sim.dof_props
        self.thormang_pose_np = thormang_pose(self.cfg, self.dof_name_to_id)
        self.thormang_pose = torch.from_numpy(self.thormang_pose_np).to(self.device)

    def _make_buffers(self) -> abi.tg_gogoro_buffers:
        b = abi.tg_gogoro_buffers()
        pairs = dict(obs_buf=self.obs_buf, rew_buf=self.rew_buf, reset_buf=self.reset_buf,
                     progress_buf=self.progress_buf, timeout_buf=self.timeout_buf, action_history=self.action_history,
                     curent_command=self.curent_command, yaw_command=self.yaw_command, curent_speed=self.curent_speed,
                     steer_offsets=self.steer_offsets, imu_offsets=self.imu_offsets,
                     speed_offset=self.curent_speed_offset, config_vector=self.config_vector,
                     buffer_obs=self.buffer_obs, thormang_pose=self.thormang_pose, root_reset=self.root_reset_tensor,
                     root=self.sim.root_state, dof_state=self.sim.dof_state, pos_target=self.sim.dof_pos_target,
                     vel_target=self.sim.dof_vel_target, dof_props=self.sim.dof_props, env_dirty=self.sim.env_dirty)
        for k, t in pairs.items():
            if not t.is_contiguous() or t.device != torch.device(self.device):
                raise RuntimeError(f"task buffer {k} must be contiguous on {self.device}")
            setattr(b, k, t.data_ptr())
        self._buf_tensors = pairs
        return b

    def _counter(self) -> int:
        self._rng_counter += 1
        return self._rng_counter

    def _dev(self, a):
        dev = self.sim.device if hasattr(self, "sim") else self.device
        return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=dev)

    # ------------------------------------------------------------ hot path
    def pre_physics_step(self, actions):
        a = actions.to(device=self.device, dtype=torch.float32).contiguous()
        draws = self._dev(self.draw_source.normal(self.n_envs)) if self.draw_source is not None else None
        check(lib().tg_gogoro_pre_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a),
                                          _p(draws), self._counter()), "tg_gogoro_pre_physics")
        self._keep = (a, draws)

    def post_physics_step(self):
        keep = None
        if self.draw_source is not None:
            ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1).cpu().numpy()
            rd, od, sd, yd = post_draws(self.draw_source, ids, self.progress_buf.cpu().numpy(),
                                        int(self.params.speed_freq_update), int(self.params.yaw_freq_update))
            keep = [self._dev(x) for x in (rd, od, sd, yd)]
        rd, od, sd, yd = keep if keep is not None else (None, None, None, None)
        check(lib().tg_gogoro_post_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(rd), _p(od),
                                           _p(sd), _p(yd), self._counter()), "tg_gogoro_post_physics")
        self._keep_post = keep
        self._post_host()

    def _post_host(self):
        """Host-side tail of post_physics_step (step count, periodic non-env DR)."""
        self.curent_step += 1
        # non-env DR (gravity every `frequency` frames, gogoro_new.py:476 -> vec_task.py:559)
        freq = self.randomization_params.get("frequency", 1)
        if self.frame_count - self.last_rand_step >= freq:
            self.apply_randomizations(self.randomization_params)

    def compute_obs_rwd(self):
        """Fused into post_physics_step (tg_gogoro_post_physics); kept for API parity."""
        raise NotImplementedError("compute_obs_rwd runs inside the fused post-physics kernel")

    def _replays_physics(self) -> bool:
        """A subclass that replaces ``simulate`` (a recorded-physics replay)
        keeps the reference's call sequence pre -> simulate -> post."""
        return type(self).simulate is not VecTask.simulate

    def step(self, actions):
        if self.dr_randomizations.get("actions", None) or self.dr_randomizations.get("observations", None):
            return super().step(actions)
        if self._replays_physics():
            self.pre_physics_step(actions)
            for _ in range(self.control_freq_inv):
                self.simulate()
            self.post_physics_step()
        else:
            # pre_physics_step + control_freq_inv x simulate + post_physics_step in
            # one library call (tg_gogoro_step: with one simulate, one launch of
            # the step kernel, the pre-physics at its start and the post-physics
            # as its epilogue); the same counters as the separate calls, and with
            # a draw_source the reference's draws in its call order (pre, then
            # post: the resets are known before the step, reset_buf)
            a = actions.to(device=self.device, dtype=torch.float32).contiguous()
            draws = (None,) * 5
            if self.draw_source is not None:
                pre = self._dev(self.draw_source.normal(self.n_envs))
                ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1).cpu().numpy()
                post = post_draws(self.draw_source, ids, self.progress_buf.cpu().numpy(),
                                  int(self.params.speed_freq_update), int(self.params.yaw_freq_update))
                draws = (pre,) + tuple(self._dev(x) for x in post)
            c_pre = self._counter()
            c_post = self._counter()
            check(lib().tg_gogoro_step(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a),
                                       self.control_freq_inv, *[_p(d) for d in draws], c_pre, c_post),
                  "tg_gogoro_step")
            self._keep = (a, draws)
            self.frame_count += self.control_freq_inv
            self._post_host()
        self.extras["time_outs"] = self.timeout_buf
        self.obs_dict["obs"] = self.obs_buf
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self._rl_out()

    # ------------------------------------------------------------ resets / draws
    def get_randoms(self, shape, bounds):
        u = self._dev(self.draw_source.uniform(shape)) if self.draw_source is not None else \
            torch.rand(shape, device=self.device)
        return bounds[0] + u * (bounds[1] - bounds[0])

    def get_randoms_norm(self, shape, mean_cov):
        r = self._dev(self.draw_source.normal(shape)) if self.draw_source is not None else \
            torch.randn(shape, device=self.device)
        return mean_cov[0] + r * mean_cov[1]

    def reset_idx(self, env_ids):
        env_ids = torch.as_tensor(env_ids, device=self.device)
        n = int(env_ids.numel())
        if n == 0:
            return
        ids32 = env_ids.to(torch.int32).contiguous()
        rd = None
        if self.draw_source is not None:
            rd = self._dev(reset_draws(self.draw_source, np.sort(env_ids.cpu().numpy()), self.n_envs))
        check(lib().tg_gogoro_reset_idx(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(ids32), n,
                                        _p(rd), self._counter()), "tg_gogoro_reset_idx")
        self._keep_reset = (ids32, rd)

"""Thormang3 flat-ground walking task (registered as "ThormangWalk").

The reference contains no Thormang walking task:
``thormang3.urdf`` is only ridden passively on the scooter and the humanoid
tasks are ``tasks/humanoid.py`` (MJCF) and the stub ``tasks/MA_OP3.py``.  This
task is designed on those patterns -- PD position control with
``control.{stiffness,damping,actionScale}`` and ``defaultJointAngles``
(cfg/task/MA_OP3.yaml:36-60), velocity-command tracking rewards
(MA_OP3.yaml:72-91), DR schema of vec_task.apply_randomizations -- and is
PARITY UNPINNED against the reference.  Its fused kernels (include/tg_walk.h)
are checked against their CPU restatement (oracle/walk_task.c).

Model: thormang3.urdf (44 links, 33 revolute DOFs) with the mesh-derived link
inertias scooter_V13.urdf carries and the xacro's foot boxes
(model/build_models.py); ``env.asset.wholeBodyCollision: true`` adds the
xacro's shin and hand boxes (model ``thormang_wb``).  Actions [N,33] in [-1,1] -> joint targets
default + actionScale * a; observation [N,112] (tg_walk.h).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from .. import abi
from .._lib import check, lib
from ..sim import load_model
from .base.vec_task import VecTask


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class ThormangWalk(VecTask):
    #: the walk's template task (MA_OP3) derives from multi_vec_task.MA_VecTask,
    #: whose __parse_sim_params sets contact_offset 0.016 before the cfg keys
    #: (multi_vec_task.py:322)
    default_contact_offset = 0.016
    #: optional DrawSource (uniform(n)/normal(n)) replacing the in-kernel Philox draws
    draw_source = None

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture, force_render):
        self.cfg = cfg
        self.model = load_model(walk_model_name(cfg))
        D = self.model.num_dof
        cfg["env"]["numObservations"] = abi_num_obs = 13 + 3 * D
        cfg["env"]["numActions"] = D
        self.num_obs_walk = abi_num_obs
        self._rng_counter = 1
        seed = cfg.get("seed", 42)
        self.seed = int(seed) if isinstance(seed, (int, float)) and seed >= 0 else 42
        super().__init__(config=cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        env = cfg["env"]
        N = self.num_envs
        dev = self.device
        self.dt = float(cfg["sim"]["dt"]) * self.control_freq_inv
        self.max_episode_length = int(math.ceil(env.get("episodeLength_s", 20) / self.dt))
        self.root_tensor = self.sim.root_state
        self.state_dof = self.sim.dof_state
        self.dof_pos = self.state_dof.view(N, D, 2)[..., 0]
        self.dof_vel = self.state_dof.view(N, D, 2)[..., 1]
        self.actions = torch.zeros(N, D, device=dev)
        self.last_actions = torch.zeros(N, D, device=dev)
        self.commands = torch.zeros(N, 3, device=dev)
        self.root_tensor[:, 2] = float(env.get("spawnHeight", 0.79))
        self.root_reset_tensor = self.root_tensor.clone()
        self.params = self._params()
        learn = env.get("learn", {})
        push_s = float(learn.get("pushInterval_s", 0.0))
        self.push_enabled = push_s > 0 and float(learn.get("pushForce", 0.0)) > 0
        self._bufs = self._make_buffers()
        self.reset_idx(torch.arange(N, device=dev))

    # ------------------------------------------------------------ creation
    def create_sim(self):
        env = self.cfg["env"]
        ao = walk_asset_options(self.cfg)
        self.sim = self.create_sim_object(self.model, ao, env_spacing=float(env.get("envSpacing", 1.0)))
        m = self.model
        self.num_dof = m.num_dof
        self.dof_names = list(m.dof_names)
        self.dof_name_to_id = m.dof_name_to_id()
        self.num_bodies = m.num_bodies
        props, self.kp, self.default_dof_pos = walk_dof_props(m, self.cfg, self.num_envs)
        self.sim.dof_props.copy_(torch.from_numpy(props))
        self.sim.env_dirty.fill_(1)
        if self.cfg["task"].get("randomize", False):
            self.apply_randomizations(self.cfg["task"]["randomization_params"])

    def _params(self) -> abi.tg_walk_params:
        return walk_params(self.cfg, self.model, self.num_envs, self.sim.G, self.dt, self.max_episode_length,
                           float(self.clip_actions), float(self.clip_obs), self.kp, self.default_dof_pos, self.seed)

    def _make_buffers(self) -> abi.tg_walk_buffers:
        b = abi.tg_walk_buffers()
        pairs = dict(obs_buf=self.obs_buf, rew_buf=self.rew_buf, reset_buf=self.reset_buf,
                     progress_buf=self.progress_buf, timeout_buf=self.timeout_buf, actions=self.actions,
                     last_actions=self.last_actions, commands=self.commands, root_reset=self.root_reset_tensor,
                     root=self.sim.root_state, dof_state=self.sim.dof_state, pos_target=self.sim.dof_pos_target,
                     body_force=self.sim.body_force if self.push_enabled else None, env_dirty=self.sim.env_dirty)
        for k, t in pairs.items():
            setattr(b, k, None if t is None else t.data_ptr())
        self._buf_tensors = pairs
        return b

    def _counter(self):
        self._rng_counter += 1
        return self._rng_counter

    def _dev(self, a):
        return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------ hot path
    def pre_physics_step(self, actions):
        a = actions.to(device=self.device, dtype=torch.float32).contiguous()
        check(lib().tg_walk_pre_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a)),
              "tg_walk_pre_physics")
        self._keep = a
        if self.push_enabled:
            self.sim.apply_body_forces(self.sim.body_force)

    def _reset_draws(self, ids):
        D = self.num_dof
        out = np.zeros((self.num_envs, 4 + 2 * D), np.float32)
        for i in ids:
            out[i] = self.draw_source.uniform(4 + 2 * D)
        return out

    def _post_draws(self):
        """Replay draws of the coming post_physics_step (None: in-kernel Philox)."""
        if self.draw_source is None:
            return None, None
        ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1).cpu().numpy()
        rd = self._dev(self._reset_draws(ids))
        pd = self._dev(self.draw_source.uniform(3 * self.num_envs).reshape(self.num_envs, 3))
        return rd, pd

    def post_physics_step(self):
        rd, pd = self._post_draws()
        check(lib().tg_walk_post_physics(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(rd), _p(pd),
                                         self._counter()), "tg_walk_post_physics")
        self._keep_post = (rd, pd)

    def step(self, actions):
        if self.dr_randomizations.get("actions", None) or self.dr_randomizations.get("observations", None):
            return super().step(actions)
        # pre_physics_step + control_freq_inv x simulate + post_physics_step in
        # one library call (tg_walk_step: the pre-physics work rides in the
        # first simulate's compose launch); reset_buf is unchanged until the
        # post kernel, so the replay draws are taken first
        a = actions.to(device=self.device, dtype=torch.float32).contiguous()
        rd, pd = self._post_draws()
        check(lib().tg_walk_step(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(a),
                                 self.control_freq_inv, _p(rd), _p(pd), self._counter()), "tg_walk_step")
        self.frame_count += self.control_freq_inv
        self._keep, self._keep_post = a, (rd, pd)
        self.extras["time_outs"] = self.timeout_buf
        self.obs_dict["obs"] = self.obs_buf
        return self._rl_out()

    def reset_idx(self, env_ids):
        env_ids = torch.as_tensor(env_ids, device=self.device)
        n = int(env_ids.numel())
        if n == 0:
            return
        ids32 = env_ids.to(torch.int32).contiguous()
        rd = self._dev(self._reset_draws(np.sort(env_ids.cpu().numpy()))) if self.draw_source is not None else None
        check(lib().tg_walk_reset_idx(self.sim.handle, C.byref(self.params), C.byref(self._bufs), _p(ids32), n,
                                      _p(rd), self._counter()), "tg_walk_reset_idx")
        self._keep_reset = (ids32, rd)


def walk_model_name(cfg) -> str:
    """The compiled model the cfg asks for: ``thormang`` (foot boxes), or with
    ``env.asset.wholeBodyCollision`` ``thormang_wb`` (feet, shins and hands
    collide; model/build_models.py)."""
    return "thormang_wb" if cfg["env"].get("asset", {}).get("wholeBodyCollision", False) else "thormang"


def walk_asset_options(cfg) -> dict:
    ao = dict(cfg["env"].get("asset", {}))
    ao.setdefault("ground_friction", 1.0)
    return ao


def walk_dof_props(m, cfg, num_envs):
    """[TG_NUM_PROPS,N,D] PD position drives on every joint (control.stiffness/damping,
    arm/head/torso joints with armStiffness/armDamping), asset armature; plus the
    per-joint stiffness and the default joint angles."""
    env = cfg["env"]
    ctl = env.get("control", {})
    D = m.num_dof
    props = abi.default_dof_props(m, num_envs)
    kp = np.full(D, float(ctl.get("stiffness", 300.0)), np.float32)
    kd = np.full(D, float(ctl.get("damping", 10.0)), np.float32)
    for i, n in enumerate(m.dof_names):
        if "arm" in n or "head" in n or "torso" in n:
            kp[i] = float(ctl.get("armStiffness", kp[i]))
            kd[i] = float(ctl.get("armDamping", kd[i]))
    props[abi.TG_PROP_DRIVE_MODE] = 1
    props[abi.TG_PROP_STIFFNESS] = kp
    props[abi.TG_PROP_DAMPING] = kd
    props[abi.TG_PROP_ARMATURE] = float(walk_asset_options(cfg).get("armature", 0.01))
    default = np.zeros(D, np.float32)
    dni = m.dof_name_to_id()
    for n, v in env.get("defaultJointAngles", {}).items():
        default[dni[n]] = v
    return props, kp, default


def walk_params(cfg, m, num_envs, num_groups, dt, max_episode_length, clip_actions, clip_obs, kp, default,
                seed) -> abi.tg_walk_params:
    env = cfg["env"]
    learn = env.get("learn", {})
    rng = env.get("randomCommandVelocityRanges", {})
    D = m.num_dof
    p = abi.tg_walk_params()
    p.num_envs, p.num_dof, p.num_obs, p.num_groups = num_envs, D, 13 + 3 * D, num_groups
    p.action_scale = float(env.get("control", {}).get("actionScale", 0.5))
    p.clip_actions = clip_actions
    p.clip_obs = clip_obs
    p.lin_vel_scale = float(learn.get("linearVelocityScale", 2.0))
    p.ang_vel_scale = float(learn.get("angularVelocityScale", 0.25))
    p.dof_pos_scale = float(learn.get("dofPositionScale", 1.0))
    p.dof_vel_scale = float(learn.get("dofVelocityScale", 0.05))
    p.cmd_vx[:] = rng.get("linear_x", [0.0, 0.6])
    p.cmd_vy[:] = rng.get("linear_y", [-0.2, 0.2])
    p.cmd_wz[:] = rng.get("yaw", [-0.5, 0.5])
    p.rew_lin_vel_xy = float(learn.get("linearVelocityXYRewardScale", 1.0))
    p.rew_ang_vel_z = float(learn.get("angularVelocityZRewardScale", 0.5))
    p.rew_upright = float(learn.get("uprightRewardScale", 0.2))
    p.rew_alive = float(learn.get("aliveReward", 0.5))
    p.rew_height = float(learn.get("heightRewardScale", 0.3))
    p.rew_action_rate = float(learn.get("actionRateRewardScale", -0.01))
    p.rew_dof_vel = float(learn.get("dofVelocityRewardScale", -1e-4))
    p.rew_torque = float(learn.get("torqueRewardScale", -2.5e-6))
    p.rew_termination = float(learn.get("terminationReward", -10.0))
    p.target_height = float(learn.get("targetHeight", 0.78))
    p.termination_height = float(learn.get("terminationHeight", 0.5))
    p.termination_up = float(learn.get("terminationUp", 0.5))
    p.spawn_height = float(env.get("spawnHeight", 0.79))
    p.joint_noise = float(env.get("jointNoise", 0.05))
    push_s = float(learn.get("pushInterval_s", 0.0))
    p.push_force = float(learn.get("pushForce", 0.0)) if push_s > 0 else 0.0
    p.push_interval = max(1, int(round(push_s / dt))) if push_s > 0 else 0
    p.max_episode_length = int(max_episode_length)
    p.dt = float(dt)
    p.default_pos[:D] = [float(x) for x in default]
    p.stiffness[:D] = [float(x) for x in kp]
    p.seed = int(seed)
    return p

"""ctypes mirrors of the C-ABI structs in include/tgsim.h and include/tg_gogoro.h,
plus the flattening of a compiled ``Model`` into a ``tg_model_desc``.

Pure data definitions: importing this module loads no library, so the CPU
tests can share the layouts with the oracle (oracle/*.c) and the product
library (libtgsim.so) alike."""
from __future__ import annotations

import ctypes as C
import hashlib
import math
from typing import Dict

import numpy as np

from .model.urdf import JOINT_FIXED, Model

P_I32 = C.POINTER(C.c_int32)
P_F32 = C.POINTER(C.c_float)
P_U8 = C.POINTER(C.c_uint8)
P_I64 = C.POINTER(C.c_int64)

TG_PROP_STIFFNESS, TG_PROP_DAMPING, TG_PROP_EFFORT, TG_PROP_VELOCITY = 0, 1, 2, 3
TG_PROP_LOWER, TG_PROP_UPPER, TG_PROP_DRIVE_MODE, TG_PROP_ARMATURE = 4, 5, 6, 7
TG_NUM_PROPS = 8
SHAPE_KIND = {"torus": 0, "box": 1, "sphere": 2}


class tg_model_desc(C.Structure):
    _fields_ = [
        ("num_links", C.c_int32), ("num_dofs", C.c_int32), ("num_groups", C.c_int32), ("num_shapes", C.c_int32),
        ("link_parent", P_I32), ("link_group", P_I32), ("link_dof", P_I32), ("link_jtype", P_I32),
        ("link_origin", P_F32), ("link_axis", P_F32), ("link_inertia", P_F32),
        ("group_root", P_I32), ("group_parent", P_I32), ("dof_locked", P_I32),
        ("shape_link", P_I32), ("shape_kind", P_I32), ("shape_pose", P_F32), ("shape_params", P_F32),
        ("shape_friction", P_F32), ("model_hash", C.c_uint64),
    ]


class tg_sim_params(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("substeps", C.c_int32), ("gravity", C.c_float * 3),
        ("linear_damping", C.c_float), ("angular_damping", C.c_float),
        ("max_depenetration_velocity", C.c_float), ("rest_offset", C.c_float), ("contact_margin", C.c_float),
        ("ground_friction", C.c_float), ("baumgarte", C.c_float), ("limit_stiffness", C.c_float),
        ("limit_damping", C.c_float), ("contact_iterations", C.c_int32),
        ("velocity_iterations", C.c_int32), ("fix_base", C.c_int32),
        ("env_spacing", C.c_float), ("envs_per_row", C.c_int32), ("solver_type", C.c_int32),
        ("contact_offset", C.c_float),
    ]


class tg_state_view(C.Structure):
    _fields_ = [
        ("root_state", C.c_void_p), ("dof_state", C.c_void_p), ("dof_pos_target", C.c_void_p),
        ("dof_vel_target", C.c_void_p), ("dof_actuation", C.c_void_p), ("dof_props", C.c_void_p),
        ("body_force", C.c_void_p), ("env_origin", C.c_void_p), ("env_dirty", C.c_void_p),
        ("num_envs", C.c_int32), ("num_dofs", C.c_int32), ("num_groups", C.c_int32), ("num_links", C.c_int32),
    ]


F2 = C.c_float * 2


class tg_gogoro_params(C.Structure):
    _fields_ = [
        ("max_steering", C.c_float), ("max_steering_change", C.c_float),
        ("steering_action_noise", F2), ("imu_filter_noise", F2), ("imu_noise", F2), ("speed_sensor_noise", F2),
        ("speed_range", F2), ("steering_offset", F2), ("speed_sensor_offset", F2),
        ("seat_offset_x_range", F2), ("seat_offset_y_range", F2), ("seat_offset_z_range", F2),
        ("seat_offset_xr_range", F2), ("steering_damping_range", F2),
        ("spawn_z", C.c_float), ("steer_stiffness", C.c_float), ("steer_effort", C.c_float),
        ("steer_velocity", C.c_float), ("clip_obs", C.c_float), ("clip_actions", C.c_float),
        ("max_episode_length", C.c_int64), ("speed_freq_update", C.c_int32), ("yaw_freq_update", C.c_int32),
        ("num_envs", C.c_int32), ("num_dof", C.c_int32),
        ("dof_steer", C.c_int32), ("dof_rear", C.c_int32), ("dof_base_x", C.c_int32), ("dof_base_y", C.c_int32),
        ("dof_base_z", C.c_int32), ("terrain_spawn", C.c_int32),
        ("absolute_steer", C.c_int32), ("debug_start_speed", C.c_int32), ("seed", C.c_uint64),
    ]


class tg_gogoro_buffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "obs_buf", "rew_buf", "reset_buf", "progress_buf", "timeout_buf",
        "action_history", "curent_command", "yaw_command", "curent_speed", "steer_offsets", "imu_offsets",
        "speed_offset", "config_vector", "buffer_obs", "thormang_pose", "root_reset",
        "root", "dof_state", "pos_target", "vel_target",
        "dof_props", "env_dirty")]


class tg_paper_params(C.Structure):
    """include/tg_gogoro_paper.h"""
    _fields_ = [
        ("num_envs", C.c_int32), ("num_dof", C.c_int32), ("num_groups", C.c_int32),
        ("dof_steer", C.c_int32), ("dof_rear", C.c_int32), ("dof_base_x", C.c_int32), ("dof_base_y", C.c_int32),
        ("dof_base_z", C.c_int32), ("max_episode_length", C.c_int64),
        ("speed_freq_update", C.c_int32), ("yaw_freq_update", C.c_int32),
        ("command_delay", F2), ("imu_filter_noise", F2), ("imu_noise", F2), ("speed_sensor_noise", F2),
        ("speed_sensor_offset", F2), ("imu_x_offset", F2), ("speed_range", F2), ("steering_offset", F2),
        ("steering_damping_range", F2), ("seat_offset_x_range", F2), ("seat_offset_y_range", F2),
        ("seat_offset_z_range", F2),
        ("max_steering", C.c_float), ("max_tilt", C.c_float), ("spawn_z", C.c_float), ("start_speed", C.c_float),
        ("push_force", C.c_float), ("push_interval", C.c_int32), ("push_max_envs", C.c_int32),
        ("use_steer_delay", C.c_int32), ("random_damping", C.c_int32), ("center_robot", C.c_int32),
        ("push_robot", C.c_int32), ("debug_start_speed", C.c_int32),
        ("damping_stiffness", C.c_float), ("damping_effort", C.c_float), ("damping_velocity", C.c_float),
        ("head_com", C.c_float * 3), ("group0_com", C.c_float * 3), ("perturbation_stride", C.c_int32),
        ("seed", C.c_uint64),
    ]


class tg_paper_buffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "obs_buf", "buffer_obs", "buffer_obs_noisy", "rew_buf", "reset_buf", "progress_buf", "timeout_buf",
        "curent_command", "command_history", "steer_delay", "steer_offsets", "curent_speed", "curent_speed_offset",
        "curent_imu_x_offset", "curent_damping_cfg", "yaw_command", "speed_no_noise", "perturbation", "root_reset",
        "thormang_pose", "root", "dof_state", "pos_target", "vel_target", "dof_props", "body_force", "env_dirty",
        "scratch", "rb_forces")]


TG_WALK_MAX_DOF = 40
F40 = C.c_float * TG_WALK_MAX_DOF


class tg_walk_params(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("num_dof", C.c_int32), ("num_obs", C.c_int32), ("num_groups", C.c_int32),
        ("action_scale", C.c_float), ("clip_actions", C.c_float), ("clip_obs", C.c_float),
        ("lin_vel_scale", C.c_float), ("ang_vel_scale", C.c_float), ("dof_pos_scale", C.c_float),
        ("dof_vel_scale", C.c_float), ("cmd_vx", F2), ("cmd_vy", F2), ("cmd_wz", F2),
        ("rew_lin_vel_xy", C.c_float), ("rew_ang_vel_z", C.c_float), ("rew_upright", C.c_float),
        ("rew_alive", C.c_float), ("rew_action_rate", C.c_float), ("rew_dof_vel", C.c_float),
        ("rew_torque", C.c_float), ("rew_termination", C.c_float), ("rew_height", C.c_float),
        ("target_height", C.c_float), ("termination_height", C.c_float), ("termination_up", C.c_float),
        ("spawn_height", C.c_float), ("joint_noise", C.c_float), ("push_force", C.c_float),
        ("push_interval", C.c_int32), ("max_episode_length", C.c_int64), ("dt", C.c_float),
        ("default_pos", F40), ("stiffness", F40), ("seed", C.c_uint64),
    ]


class tg_walk_buffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "obs_buf", "rew_buf", "reset_buf", "progress_buf", "timeout_buf", "actions", "last_actions", "commands",
        "root_reset", "root", "dof_state", "pos_target", "body_force", "env_dirty")]


def model_arrays(m: Model) -> Dict[str, np.ndarray]:
    """Flatten a grouped Model into the tg_model_desc arrays (numpy, C-contiguous)."""
    L, D, G, S = m.num_bodies, m.num_dof, m.num_groups, len(m.shapes)
    a = {
        "link_parent": np.array([l.parent for l in m.links], np.int32),
        "link_group": np.array(m.link_group, np.int32),
        "link_dof": np.array([m.joints[l.joint].dof if l.joint >= 0 else -1 for l in m.links], np.int32),
        "link_jtype": np.array([m.joints[l.joint].jtype if l.joint >= 0 else JOINT_FIXED for l in m.links], np.int32),
        "link_origin": np.zeros((L, 12), np.float32),
        "link_axis": np.zeros((L, 3), np.float32),
        "link_inertia": np.zeros((L, 10), np.float32),
        "group_root": np.array(m.group_root, np.int32),
        "group_parent": np.array(m.group_parent, np.int32),
        "dof_locked": np.zeros(D, np.int32),
        "shape_link": np.array([m.link_index(s.link) for s in m.shapes], np.int32).reshape(S),
        "shape_kind": np.array([SHAPE_KIND[s.kind] for s in m.shapes], np.int32).reshape(S),
        "shape_pose": np.zeros((S, 12), np.float32),
        "shape_params": np.zeros((S, 4), np.float32),
        "shape_friction": np.array([s.friction for s in m.shapes], np.float32).reshape(S),
    }
    for i, l in enumerate(m.links):
        if l.joint >= 0:
            j = m.joints[l.joint]
            a["link_origin"][i, :9] = np.asarray(j.origin_rot).reshape(9)
            a["link_origin"][i, 9:] = j.origin_pos
            a["link_axis"][i] = j.axis
        else:
            a["link_origin"][i, :9] = np.eye(3).reshape(9)
        a["link_inertia"][i] = [l.mass, *l.com, *l.inertia]
    a["dof_locked"][m.locked_dofs] = 1
    for i, s in enumerate(m.shapes):
        a["shape_pose"][i, :9] = np.asarray(s.rot).reshape(9)
        a["shape_pose"][i, 9:] = s.pos
        a["shape_params"][i, :len(s.params)] = s.params
    return a


def model_hash(arrays: Dict[str, np.ndarray]) -> int:
    h = hashlib.sha1()
    for k in sorted(arrays):
        h.update(k.encode())
        h.update(np.ascontiguousarray(arrays[k]).tobytes())
    return int.from_bytes(h.digest()[:8], "little")


class ModelDesc:
    """Owns the numpy arrays behind a tg_model_desc."""

    def __init__(self, m: Model):
        self.model = m
        self.arrays = model_arrays(m)
        self.hash = model_hash(self.arrays)
        d = tg_model_desc()
        d.num_links, d.num_dofs, d.num_groups, d.num_shapes = m.num_bodies, m.num_dof, m.num_groups, len(m.shapes)
        for k, v in self.arrays.items():
            ptype = P_I32 if v.dtype == np.int32 else P_F32
            setattr(d, k, v.ctypes.data_as(ptype))
        d.model_hash = self.hash
        self.desc = d


def default_dof_props(m: Model, num_envs: int) -> np.ndarray:
    """[TG_NUM_PROPS, N, D] initial per-env DOF properties, as gym.get_asset_dof_properties
    reports them for a URDF (drive mode none, zero gains, URDF limits/effort/velocity)."""
    D = m.num_dof
    p = np.zeros((TG_NUM_PROPS, D), np.float32)
    for d, ji in enumerate(m.dof_joint):
        j = m.joints[ji]
        p[TG_PROP_LOWER, d] = j.lower if j.has_limits else -3.4e38
        p[TG_PROP_UPPER, d] = j.upper if j.has_limits else 3.4e38
        p[TG_PROP_EFFORT, d] = j.effort
        p[TG_PROP_VELOCITY, d] = j.velocity
    return np.repeat(p[:, None, :], num_envs, axis=1)


#: physx keys that size PhysX's own thread pool / GPU buffers: no effect on the
#: simulated result there either, accepted silently
PHYSX_RESOURCE_KEYS = frozenset({
    "num_threads", "num_subscenes", "use_gpu", "default_buffer_size_multiplier", "max_gpu_contact_pairs",
    "contact_collection"})
#: physx keys honoured by the solver (DESIGN.md §4 "Solver cfg"); solver_type
#: 0 (PGS) and 1 (TGS) are both implemented, other values warn
PHYSX_HONOURED_KEYS = frozenset({"num_position_iterations", "num_velocity_iterations", "rest_offset",
                                 "max_depenetration_velocity", "contact_offset"})
#: physx keys that cannot change a result of these tasks in PhysX either:
#: bounce_threshold_velocity only gates restitution, and every material here
#: (and in the reference, which sets none) has restitution 0
PHYSX_INERT_KEYS = frozenset({"bounce_threshold_velocity"})


class SolverCfgWarning(UserWarning):
    """A cfg ``sim.physx`` key whose PhysX meaning the contact solver does not reproduce."""


def unhonoured_physx_keys(physx: dict, asset_opts: dict | None = None) -> Dict[str, str]:
    """The ``sim.physx`` keys (``vec_task.py:470-482`` sets them on PhysX's
    params) that would change a PhysX result but not this solver's, each with
    the reason.  ``solver_type`` 0 (PGS) and 1 (TGS, the position iterations
    as sub-steps with re-formed contact targets, DESIGN.md §4 "Solver cfg")
    are honoured, any other value is reported; ``contact_offset`` is honoured
    since round 5 (round 6: PhysX's pair rule -- a point's normal row exists
    only while its separation is below the shape's plus the ground plane's
    offset, 2 x ``tg_sim_params.contact_offset``);
    ``bounce_threshold_velocity`` is inert (``PHYSX_INERT_KEYS``).  Unknown
    keys are reported too."""
    ao = asset_opts or {}
    out: Dict[str, str] = {}
    for k, v in physx.items():
        if k in PHYSX_RESOURCE_KEYS or k in PHYSX_HONOURED_KEYS or k in PHYSX_INERT_KEYS:
            continue
        if k == "solver_type":
            if int(v) not in (0, 1):
                out[k] = f"{v} is neither PGS (0) nor TGS (1); TGS is used"
        else:
            out[k] = "unknown physx key, ignored"
    return out


def sim_params_from_cfg(cfg_sim: dict, asset_opts: dict | None = None, num_envs: int = 1,
                        env_spacing: float = 1.0, warn: bool = True,
                        default_contact_offset: float = 0.02) -> tg_sim_params:
    """Map the reference cfg 'sim' block (vec_task.py:442-490) onto tg_sim_params.

    ``num_position_iterations`` is the number of biased PGS sweeps per substep
    (an asset option ``contact_iterations`` overrides it),
    ``num_velocity_iterations`` the bias-free sweeps after them (asset option
    ``velocity_iterations``); the physx keys the
    solver does not reproduce raise one ``SolverCfgWarning`` naming each
    (``unhonoured_physx_keys``)."""
    import warnings
    physx = cfg_sim.get("physx", {})
    if warn:
        bad = unhonoured_physx_keys(physx, asset_opts)
        if bad:
            warnings.warn("sim.physx keys not reproduced by the contact solver: " +
                          "; ".join(f"{k}: {r}" for k, r in bad.items()), SolverCfgWarning, stacklevel=2)
    ao = asset_opts or {}
    sp = tg_sim_params()
    sp.dt = float(cfg_sim["dt"])
    sp.substeps = int(cfg_sim.get("substeps", 2))
    sp.gravity[:] = [float(x) for x in cfg_sim.get("gravity", [0.0, 0.0, -9.81])]
    sp.linear_damping = float(ao.get("linear_damping", 0.0))
    sp.angular_damping = float(ao.get("angular_damping", 0.5))
    sp.max_depenetration_velocity = float(physx.get("max_depenetration_velocity", 100.0))
    sp.rest_offset = float(physx.get("rest_offset", 0.001))
    sp.contact_margin = float(ao.get("contact_margin", 0.05))
    # contact_offset: the cfg's sim.physx key.  Without it, the default of the
    # VecTask base the task derives from: vec_task.py:442-482 leaves IsaacGym's
    # own 0.02 (Gogoro), multi_vec_task.py:322 sets 0.016 before the cfg keys
    # (the MA_OP3 template of the walk), passed in by the task as
    # ``default_contact_offset``.  <= 0 keeps every point speculative
    sp.contact_offset = float(physx.get("contact_offset", default_contact_offset))
    sp.ground_friction = float(ao.get("ground_friction", 1.0))
    sp.baumgarte = float(ao.get("baumgarte", 0.2))
    sp.limit_stiffness = float(ao.get("limit_stiffness", 1.0))
    sp.limit_damping = float(ao.get("limit_damping", 1.0))
    sp.contact_iterations = int(ao.get("contact_iterations", max(1, int(physx.get("num_position_iterations", 4)))))
    # IsaacGym's default num_velocity_iterations is 1; an asset option overrides it
    sp.velocity_iterations = int(ao.get("velocity_iterations", max(0, int(physx.get("num_velocity_iterations", 1)))))
    # IsaacGym's default solver_type is 1 (TGS)
    sp.solver_type = 0 if int(physx.get("solver_type", 1)) == 0 else 1
    sp.fix_base = int(bool(ao.get("fix_base_link", False)))
    sp.env_spacing = float(env_spacing)
    sp.envs_per_row = max(1, int(math.sqrt(num_envs)))
    return sp

"""Oracle env for the Gogoro "paper" variant (test infrastructure).

``OraclePaper`` drives oracle/gogoro_paper_task.c exactly like the product
class thormang_isaacgym_amd.tasks.gogoro_paper.Gogoro drives the HIP kernels:
same parameter block, same per-env draw arrays (tasks/paper_draws.py).  The
physics is either replayed from a fixture or the fp64 oracle engine."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from tests.oracle_lib import lib, physics_step, ptr
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.model.urdf import Model
from thormang_isaacgym_amd.tasks.gogoro_paper import ASSET_OPTIONS, paper_dof_props, paper_params, paper_pose
from thormang_isaacgym_amd.tasks.paper_draws import ctor_draws, post_draws, reset_draws

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ("DEBUGFIXBASE", "DEBUG_START_SPEED", "RANDOM_DAMPING", "PUSH_ROBOT", "CENTER_ROBOT", "USE_STEER_DELAY")


def load_v12():
    with open(os.path.join(REPO, "thormang_isaacgym_amd", "model", "compiled", "gogoro_v12.json")) as f:
        return Model.from_json(f.read())


def switches_from(flags) -> dict:
    sw = {k: bool(v) for k, v in zip(FLAGS, flags)}
    sw["DEBUGUSETERRAIN"] = False
    return sw


def fixture_cfg(f):
    from tests.golden.make_golden_paper import paper_cfg
    return paper_cfg(int(f["n_envs"]), int(f["max_steps"]), int(f["freq"]))


class OraclePaper:
    def __init__(self, cfg, draws, switches, root_origins=None, threads=8, precision="f64"):
        self.cfg, self.src, self.sw, self.threads = cfg, draws, switches, threads
        self.L = lib(precision)   # f32: the rounding control of the TGS parity tests
        self.model = m = load_v12()
        self.n = n = cfg["env"]["numEnvs"]
        self.D = D = m.num_dof
        self.p = paper_params(cfg, m, n, switches)
        z = lambda *s, dt=np.float32: np.zeros(s, dt)
        u = ctor_draws(draws, n)
        nz = cfg["noises"]
        aff = lambda c, b: (np.float32(b[0]) + u[:, c] * np.float32(b[1] - b[0])).astype(np.float32)
        self.a = a = dict(
            obs_buf=z(n, 160), buffer_obs=z(n, 20, 8), buffer_obs_noisy=z(n, 20, 8), rew_buf=z(n),
            reset_buf=np.ones(n, np.int64), progress_buf=z(n, dt=np.int64), timeout_buf=z(n, dt=np.uint8),
            curent_command=z(n), command_history=z(n, 5),
            steer_delay=aff(2, nz["command_delay"]).astype(np.int64),
            steer_offsets=aff(1, nz["steering_offset"]), curent_speed=aff(0, nz["speed_range"]),
            curent_speed_offset=aff(4, nz["speed_sensor_offset"]), curent_imu_x_offset=aff(5, nz["imu_x_offset"]),
            curent_damping_cfg=aff(3, nz["steering_damping_range"]), yaw_command=z(n), speed_no_noise=z(n),
            perturbation=z(n, 3), root_reset=z(n, 13), thormang_pose=paper_pose(cfg, m.dof_name_to_id(), n),
            root=z(n, 13), dof_state=z(n * D, 2), pos_target=z(n, D), vel_target=z(n, D),
            dof_props=paper_dof_props(m, cfg, n), body_force=z(n, m.num_groups, 6), env_dirty=z(n, dt=np.uint8),
            scratch=z(n))
        if root_origins is not None:
            a["root"][:, 0:3] = root_origins
        a["root"][:, 2] = 1.0
        a["root"][:, 6] = 1.0
        a["root_reset"][:] = a["root"]
        a["root_reset"][:, 7:13] = 0
        self.b = abi.tg_paper_buffers(**{k: v.ctypes.data for k, v in a.items()})
        if not switches["PUSH_ROBOT"]:
            self.b.body_force = None
        rd = reset_draws(draws, np.arange(n), n, switches["RANDOM_DAMPING"], switches["CENTER_ROBOT"])
        for e in range(n):
            self.L.oracle_paper_reset_env(C.byref(self.p), C.byref(self.b), e, ptr(np.ascontiguousarray(rd[e])))
        self.desc = self.sp = None
        self.head_id = [l.name for l in m.links].index("head_p_link")

    def pre(self, actions):
        self.L.oracle_paper_pre_physics(C.byref(self.p), C.byref(self.b),
                                       ptr(np.ascontiguousarray(actions, np.float32)))

    def post(self):
        a = self.a
        ids = np.nonzero(a["reset_buf"])[0]
        rd, nd, sd, yd, pd = post_draws(self.src, ids, a["progress_buf"].copy(), int(self.p.speed_freq_update),
                                        self.sw["PUSH_ROBOT"], self.sw["RANDOM_DAMPING"], self.sw["CENTER_ROBOT"])
        self.L.oracle_paper_post_physics(C.byref(self.p), C.byref(self.b), ptr(rd), ptr(nd), ptr(sd), ptr(yd), ptr(pd))
        if self.sw["PUSH_ROBOT"]:   # apply_rigid_body_force_tensors of the [N*L, 3] perturbations (:449-457)
            if self.desc is None:
                self.desc = abi.ModelDesc(self.model)
            L = self.model.num_bodies
            f = np.zeros((self.n, L, 3), np.float32)
            f[:, self.head_id] = a["perturbation"]
            self._forces = f
            self.L.oracle_rigid_body_force_wrench(C.byref(self.desc.desc), self.n, ptr(a["root"]), ptr(a["dof_state"]),
                                                 None, ptr(f), None, 0, ptr(a["body_force"]))
        return a["obs_buf"], a["rew_buf"], a["reset_buf"], a["timeout_buf"]

    def step(self, actions):
        """pre -> oracle physics -> post (actions [N] or [N,1])."""
        self.pre(np.asarray(actions, np.float32).reshape(-1))
        self.physics()
        return self.post()

    def physics(self, env_spacing=1.0):
        """One control step of the fp64 oracle engine (the product's tg_simulate)."""
        if self.desc is None:
            self.desc = abi.ModelDesc(self.model)
        if self.sp is None:
            ao = dict(ASSET_OPTIONS, fix_base_link=bool(self.sw["DEBUGFIXBASE"]))
            self.sp = abi.sim_params_from_cfg(self.cfg["sim"], ao, self.n, env_spacing, warn=False)
        a = self.a
        force = a["body_force"] if self.sw["PUSH_ROBOT"] else None
        physics_step(self.desc, self.sp, a["root"], a["dof_state"], a["dof_props"], a["pos_target"], a["vel_target"],
                     force=force, threads=self.threads, L=self.L)

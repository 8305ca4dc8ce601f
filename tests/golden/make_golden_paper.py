"""Golden fixtures for the Gogoro "paper" variant.

RUNS ONLY IN THE BUILD CONTAINER (needs /root/reference).  Imports the
reference's unregistered ``isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py``
behind the same shim as make_golden.py and drives its own methods
(``pre_physics_step`` :349-393, ``post_physics_step`` :397-482,
``compute_obs_rwd`` :491-547, ``reset_idx`` :609-692, ``compute_gogoro_reward``
:714-762, ``compute_gogoro_observations`` :771-808) through
``VecTask.step`` (vec_task.py:313-359) on a synthetic physics, recording every
torch.rand draw in order.  The module's debug switches are run as committed
(DEBUG = True: fixed base, start speed, pushes, centred rider, fixed 2-step
steering delay) and once flipped (per-env delay, random steering damping,
random seat offsets, no start speed) -> paper_steps.npz / paper_steps_flags.npz.

Two reference quirks bound the fixture: ``speed_command_change[speed_command_change]``
(:405-408) raises IndexError unless the envs due for a command change are
exactly {0..k-1}, and the push mask ``progress_buf[:2048]`` (:443) only
matches the perturbation tensor for <= 2048 envs.  The synthetic physics
therefore keeps every env upright (no falls) in the runs that exercise the
command changes, and a separate run with falls uses a command period longer
than the run.

Only data is written; no reference source leaves the container.
Re-run:  python tests/golden/make_golden_paper.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from tests.golden.make_golden import DrawLog, FakeGym, REF, TorchProxy, load_reference, urdf_dof_props  # noqa: E402

import importlib.util  # noqa: E402


def load_paper():
    vt, _ = load_reference()
    spec = importlib.util.spec_from_file_location("ref_gogoro_paper",
                                                  f"{REF}/tasks/gogoro_realistic_turning_sim_paper.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ref_gogoro_paper"] = mod
    spec.loader.exec_module(mod)
    return vt, mod


def paper_cfg(n_envs, max_steps=20, freq=7):
    """cfg/task/Gogoro_paper.yaml values (noises, joints_pos); env size and the
    command period are the fixture's."""
    return {
        "name": "Gogoro",
        "env": {"numEnvs": n_envs, "max_steps": max_steps},
        "sim": {"dt": 0.03, "up_axis": "z", "use_gpu_pipeline": False, "gravity": [0.0, 0.0, -9.81], "substeps": 3},
        "noises": {
            "imu_filter_noise": [-0.003, 0.003], "imu_noise": [-0.003, 0.003], "speed_sensor_offset": [-0.3, 0.3],
            "speed_sensor_noise": [0, 0.3], "seat_offset_x_range": [-0.1, 0.1], "seat_offset_y_range": [-0.1, 0.1],
            "seat_offset_z_range": [-0.05, 0.05], "imu_x_offset": [-0.02, 0.02], "spawn_x_angle": [-0.02, 0.02],
            "steering_action_noise": [-0.05, 0.05], "steering_offset": [-0.05, 0.05], "command_delay": [0, 5],
            "steering_damping_range": [50, 1000], "IK_noise_amplitude": [0, 3], "speed_range": [5.0, 20.0],
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


class PaperGym(FakeGym):
    """FakeGym plus the force API; ``tilt`` scales the synthetic attitude walk."""

    def __init__(self, env, num_dof, rs, tilt):
        super().__init__(env, num_dof, rs)
        self.tilt = tilt
        self.forces = None

    def apply_rigid_body_force_tensors(self, sim, f, t):
        self.forces = f.clone()
        return True

    def simulate(self, sim):
        self.frame += 1
        rt = self.env.root_tensor
        n = rt.shape[0]
        # attitude: small random roll/pitch around upright (scaled), free yaw
        roll = self.rs.normal(0, 0.05 * self.tilt, n) + (self.tilt > 1.0) * np.linspace(0, 0.5, n) * self.rs.random(n)
        pitch = self.rs.normal(0, 0.02, n)
        yaw = self.rs.uniform(-np.pi, np.pi, n)
        cr, sr, cp, sp, cy, sy = (np.cos(roll / 2), np.sin(roll / 2), np.cos(pitch / 2), np.sin(pitch / 2),
                                  np.cos(yaw / 2), np.sin(yaw / 2))
        q = np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                      cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy], 1)
        rt[:, 3:7] = torch.from_numpy(q).float()
        rt[:, 7:10] = torch.from_numpy(self.rs.normal(0, 2.0, (n, 3))).float()
        rt[:, 10:13] = torch.from_numpy(self.rs.normal(0, 1.0, (n, 3))).float()
        rt[:, 0:3] += 0.03 * rt[:, 7:10]
        sd = self.env.state_dof
        sd += torch.from_numpy(self.rs.normal(0, 0.01, tuple(sd.shape))).float()


def make_env(vt, pm, cfg, fake_rs, tilt):
    """Mirror of Gogoro.__init__ (paper :35-163) minus the simulator, with the
    _create_envs dof-prop setup (:250-300) and the closing reset_idx(all)."""
    G = pm.Gogoro
    g = object.__new__(G)
    model, props = urdf_dof_props()
    g.steering_sensitivity = 0.1
    g.curent_step = 0
    g.device = "cpu"
    g.rl_device = "cpu"
    g.n_envs = n = cfg["env"]["numEnvs"]
    g.num_environments = n
    g.max_episode_length = torch.tensor(cfg["env"]["max_steps"])
    nz = cfg["noises"]
    g.imu_filter_noise, g.imu_noise = nz["imu_filter_noise"], nz["imu_noise"]
    g.speed_sensor_noise, g.speed_sensor_offset = nz["speed_sensor_noise"], nz["speed_sensor_offset"]
    g.seating_offset = torch.ones((n, 3))
    g.seat_offset_x_range, g.seat_offset_y_range = nz["seat_offset_x_range"], nz["seat_offset_y_range"]
    g.seat_offset_z_range, g.spawn_x_angle = nz["seat_offset_z_range"], nz["spawn_x_angle"]
    g.imu_x_offset, g.steering_damping_range = nz["imu_x_offset"], nz["steering_damping_range"]
    g.steering_action_noise, g.speed_range = nz["steering_action_noise"], nz["speed_range"]
    g.speed_freq_update, g.yaw_freq_update = nz["speed_freq_update"], nz["yaw_freq_update"]
    g.steering_offset, g.command_delay = nz["steering_offset"], nz["command_delay"]
    g.dof_props = None
    g.yaw_command = torch.zeros(n)
    g.min_speed, g.max_speed, g.max_steering = 0.0, 10.0, 0.5
    # draws in __init__ order (:75-90)
    g.curent_speed = g.get_randoms(n, g.speed_range)
    g.last_err = torch.zeros(n)
    g.curent_command = torch.zeros(n)
    g.steer_offsets = g.get_randoms(n, g.steering_offset)
    g.steer_delay = g.get_randoms(n, g.command_delay).to(torch.long)
    g.command_history = torch.zeros((n, g.command_delay[1]))
    g.envs_indexes_ = torch.arange(0, n)
    g.curent_damping_cfg = g.get_randoms(n, g.steering_damping_range)
    g.curent_speed_offset = g.get_randoms(n, g.speed_sensor_offset)
    g.curent_imu_x_offset = g.get_randoms(n, g.imu_x_offset)
    g.speed_no_noise = torch.zeros(n)
    g.integral_error = torch.zeros(n)
    g.last_err_speed = torch.zeros(n)
    g.viewer = None
    g.cfg = cfg
    g.buff_size = 20
    g.buffer_obs = torch.zeros((n, 20, 8))
    g.buffer_obs_noisy = torch.zeros((n, 20, 8))
    g.num_observations, g.num_actions, g.num_states = 160, 1, 0
    g.control_freq_inv = 1
    g.clip_obs, g.clip_actions = math.inf, math.inf
    g.dr_randomizations = {}
    g.force_render = False
    g.extras, g.obs_dict = {}, {}
    g.sim = None
    g.num_dof = model.num_dof
    g.dof_names = model.dof_names
    g.dof_name_to_id = {k: v for k, v in zip(g.dof_names, np.arange(g.num_dof))}
    g.num_rgbd = model.num_bodies
    g.rgid_body_to_id = {l.name: i for i, l in enumerate(model.links)}
    g.envs = list(range(n))
    g.handles = list(range(n))
    g.gym = PaperGym(g, g.num_dof, fake_rs, tilt)
    vt.VecTask.allocate_buffers(g)
    g.dof_props = props
    g.thormang_pose = torch.zeros(n, g.num_dof)
    dni = g.dof_name_to_id
    for i in range(n):
        for d in range(g.num_dof):
            g.dof_props["driveMode"][d] = 0
            g.dof_props["damping"][d] = 0.0
            g.dof_props["stiffness"][d] = 0.0
            g.dof_props["effort"][d] = 0.0
        for j_name in cfg["joints_pos"]:
            idd = dni[j_name]
            g.dof_props["lower"][idd] = cfg["joints_pos"][j_name]
            g.dof_props["upper"][idd] = g.dof_props["lower"][idd] + 0.0001
            g.thormang_pose[:, idd] = float(g.dof_props["lower"][idd] + 0.0001 / 2)
        for b in ("base_x", "base_y", "base_z"):
            g.dof_props["lower"][dni[b]] = 0.0
            g.dof_props["upper"][dni[b]] = g.dof_props["lower"][dni[b]] + 0.0001
            g.thormang_pose[i, dni[b]] = float(g.dof_props["lower"][dni[b]] + 0.0001 / 2)
        rw, st = dni["rear_wheel_joint"], dni["steering_joint"]
        g.dof_props["driveMode"][rw], g.dof_props["stiffness"][rw] = 2, 0.0
        g.dof_props["damping"][rw], g.dof_props["effort"][rw] = 1000.0, 170.0
        g.dof_props["driveMode"][st], g.dof_props["stiffness"][st] = 1, 100.0
        g.dof_props["damping"][st], g.dof_props["effort"][st], g.dof_props["velocity"][st] = 100.0, 10.0, 50.0
        g.gym.set_actor_dof_properties(i, i, g.dof_props)
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
    g.current_steering = None
    return g, model


FLAGS = ("DEBUGFIXBASE", "DEBUG_START_SPEED", "RANDOM_DAMPING", "PUSH_ROBOT", "CENTER_ROBOT", "USE_STEER_DELAY")


def run(vt, pm, n_envs, T, max_steps, freq, tilt, seed, flags=None):
    saved = {k: getattr(pm, k) for k in FLAGS}
    if flags:
        for k, v in flags.items():
            setattr(pm, k, v)
    try:
        torch.manual_seed(seed)
        fake_rs = np.random.default_rng(seed + 1)
        act_rs = np.random.default_rng(seed + 2)
        log = DrawLog()
        pm.torch = TorchProxy(log)
        cfg = paper_cfg(n_envs, max_steps, freq)
        g, model = make_env(vt, pm, cfg, fake_rs, tilt)
        n_init = len(log.kind)
        g.reset_idx(torch.arange(0, n_envs).long())
        init = dict(root=g.root_tensor.clone().numpy(), dof=g.state_dof.clone().numpy(),
                    n_draws_ctor=np.int64(n_init), n_draws_init=np.int64(len(log.kind)))
        for k in ("curent_speed", "steer_offsets", "steer_delay", "curent_damping_cfg", "curent_speed_offset",
                  "curent_imu_x_offset", "yaw_command"):
            init[k] = getattr(g, k).clone().numpy()
        keys = ("actions", "draw_end", "sim_root", "sim_dof", "obs", "rew", "reset", "time_outs", "progress",
                "curent_command", "command_history", "yaw_command", "curent_speed", "steer_offsets", "steer_delay",
                "curent_speed_offset", "curent_imu_x_offset", "buffer_obs", "buffer_obs_noisy", "pos_target",
                "vel_target", "root_after", "dof_after", "perturbation", "steer_damping", "steer_stiffness",
                "steer_effort", "steer_velocity", "seat_lower", "seat_upper", "speed_no_noise")
        rec = {k: [] for k in keys}
        orig_sim = g.gym.simulate

        def sim_and_record(sim):
            orig_sim(sim)
            rec["sim_root"].append(g.root_tensor.clone().numpy())
            rec["sim_dof"].append(g.state_dof.clone().numpy())

        g.gym.simulate = sim_and_record
        dni = g.dof_name_to_id
        st, seat = dni["steering_joint"], [dni["base_x"], dni["base_y"], dni["base_z"]]
        head = g.rgid_body_to_id["head_p_link"]
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
            for k in ("curent_command", "command_history", "yaw_command", "curent_speed", "steer_offsets",
                      "steer_delay", "curent_speed_offset", "curent_imu_x_offset", "buffer_obs", "buffer_obs_noisy",
                      "speed_no_noise"):
                rec[k].append(getattr(g, k).clone().numpy())
            rec["pos_target"].append(g.gym.pos_target.numpy())
            rec["vel_target"].append(g.gym.vel_target.numpy())
            rec["root_after"].append(g.root_tensor.clone().numpy())
            rec["dof_after"].append(g.state_dof.clone().numpy())
            rec["perturbation"].append(g.curent_perturbations[:, head].clone().numpy())
            ep = g.gym.env_props
            for k, f in (("steer_damping", "damping"), ("steer_stiffness", "stiffness"), ("steer_effort", "effort"),
                         ("steer_velocity", "velocity")):
                rec[k].append(ep[f][:, st].copy())
            rec["seat_lower"].append(ep["lower"][:, seat].copy())
            rec["seat_upper"].append(ep["upper"][:, seat].copy())
        kinds, sizes, vals = log.arrays()
        out = {k: np.stack(v) for k, v in rec.items()}
        out.update({f"init_{k}": v for k, v in init.items()})
        out.update(draw_kind=kinds, draw_size=sizes, draw_vals=vals, n_envs=np.int64(n_envs),
                   max_steps=np.int64(max_steps), freq=np.int64(freq),
                   flags=np.array([int(getattr(pm, k)) for k in FLAGS], np.int64))
        return out
    finally:
        for k, v in saved.items():
            setattr(pm, k, v)


def main():
    vt, pm = load_paper()
    flipped = dict(USE_STEER_DELAY=True, RANDOM_DAMPING=True, CENTER_ROBOT=False, DEBUG_START_SPEED=False)
    jobs = {
        # as committed: upright envs, command changes at progress 7 and 14, timeouts at 20
        "paper_steps.npz": dict(n_envs=12, T=50, max_steps=20, freq=7, tilt=1.0, seed=11),
        # falls (tilt ramp across envs), no command change inside the run
        "paper_falls.npz": dict(n_envs=12, T=40, max_steps=30, freq=1000, tilt=4.0, seed=12),
        # the module's switches flipped
        "paper_steps_flags.npz": dict(n_envs=12, T=50, max_steps=20, freq=7, tilt=1.0, seed=13, flags=flipped),
    }
    for fn, kw in jobs.items():
        out = run(vt, pm, **kw)
        np.savez_compressed(os.path.join(HERE, fn), **out)
        print(fn, os.path.getsize(os.path.join(HERE, fn)), "draws", len(out["draw_kind"]),
              "resets", int(out["reset"].sum()), "timeouts", int(out["time_outs"].sum()))


if __name__ == "__main__":
    main()

"""Env / VecTask: the IsaacGymEnvs task API on top of libtgsim.

Mirrors ``isaacgymenvs/tasks/base/vec_task.py`` of the reference (same class
names, constructor signature, buffers, ``step``/``reset``/``reset_done``
semantics, cfg keys) so ``train.py`` + rl_games drive it unchanged:

* ``Env.__init__``                  vec_task.py:61-108
* properties                        vec_task.py:139-162
* ``VecTask.__init__``              vec_task.py:169-223
* ``allocate_buffers``              vec_task.py:254-277
* ``step``                          vec_task.py:313-359
* ``zero_actions/reset/reset_done`` vec_task.py:361-406
* ``__parse_sim_params``            vec_task.py:442-490 (-> abi.tg_sim_params)
* ``apply_randomizations``          vec_task.py:538-768, vectorised: gravity
  (sim_params), per-body mass scale (actor rigid_body_properties.mass),
  per-shape friction (rigid_shape_properties.friction) and the observation /
  action noise lambdas.  Sampling follows the documented IsaacGym DR
  semantics (uniform / gaussian / loguniform, additive / scaling, schedules);
  the exact RNG stream of the absent ``dr_utils`` is not reproducible
  (parity unpinned).

Viewer/rendering is out of scope: ``headless=False`` runs
headless with a warning.  The CPU pipeline runs its physics on the GPU and
delivers the step tensors on rl_device (``pipeline_device``).
"""
from __future__ import annotations

import abc
import math
import operator
import warnings
from typing import Any, Dict, Tuple

import numpy as np
import torch

from ... import abi


class _Box:
    """Minimal stand-in for ``gym.spaces.Box`` (gym is not a dependency): rl_games
    reads ``.shape``, ``.low``, ``.high``."""

    def __init__(self, low, high):
        self.low = np.asarray(low, np.float32)
        self.high = np.asarray(high, np.float32)
        self.shape = self.low.shape
        self.dtype = np.float32

    def __repr__(self):
        return f"Box({self.shape})"


def _space(low, high):
    try:
        from gym import spaces  # noqa: WPS433
        return spaces.Box(low, high)
    except Exception:
        return _Box(low, high)


def pipeline_device(config: Dict[str, Any], sim_device: str) -> str:
    """The GPU the env state and kernels live on.  The reference's GPU pipeline
    (vec_task.py:66-74: sim_device 'cuda:N', use_gpu_pipeline) maps to cuda:N.
    Its CPU pipeline (BASELINE config 1: sim_device=cpu, pipeline=cpu) has no
    CPU physics here -- libtgsim simulates on an MI355X -- so the env runs on
    cuda:N (N from sim_device, else 0) and VecTask delivers the step tensors
    on rl_device; without a GPU this raises (the CPU engine under oracle/ is
    test infrastructure, never a fallback)."""
    dev_type, _, idx = sim_device.partition(":")
    gpu_pipeline = bool(config["sim"].get("use_gpu_pipeline", True)) and dev_type.lower() in ("cuda", "gpu")
    if not gpu_pipeline:
        if not torch.cuda.is_available():
            raise RuntimeError("the CPU pipeline runs its physics on an MI355X (libtgsim has no CPU engine) "
                               "and no GPU is visible")
        warnings.warn(f"CPU pipeline requested (sim_device={sim_device!r}, use_gpu_pipeline="
                      f"{config['sim'].get('use_gpu_pipeline', True)}): physics and task kernels run on "
                      f"cuda:{int(idx) if idx else 0}, step tensors are delivered on rl_device")
    return f"cuda:{int(idx) if idx else 0}"


class Env(abc.ABC):
    def __init__(self, config: Dict[str, Any], rl_device: str, sim_device: str, graphics_device_id: int,
                 headless: bool):
        split_device = sim_device.split(":")
        self.device_type = split_device[0]
        self.device_id = int(split_device[1]) if len(split_device) > 1 else 0
        self.device = pipeline_device(config, sim_device)
        self.rl_device = rl_device
        self.headless = headless
        enable_camera_sensors = config.get("enableCameraSensors", False)
        self.graphics_device_id = graphics_device_id
        if not enable_camera_sensors and self.headless:
            self.graphics_device_id = -1
        self.num_environments = config["env"]["numEnvs"]
        self.num_agents = config["env"].get("numAgents", 1)
        self.num_observations = config["env"]["numObservations"]
        self.num_states = config["env"].get("numStates", 0)
        self.num_actions = config["env"]["numActions"]
        self.control_freq_inv = config["env"].get("controlFrequencyInv", 1)
        self.obs_space = _space(np.ones(self.num_obs) * -np.inf, np.ones(self.num_obs) * np.inf)
        self.state_space = _space(np.ones(self.num_states) * -np.inf, np.ones(self.num_states) * np.inf)
        self.act_space = _space(np.ones(self.num_actions) * -1.0, np.ones(self.num_actions) * 1.0)
        self.clip_obs = config["env"].get("clipObservations", math.inf)
        self.clip_actions = config["env"].get("clipActions", math.inf)

    @abc.abstractmethod
    def allocate_buffers(self):
        """Create torch buffers for observations, rewards, actions dones and any additional data."""

    @abc.abstractmethod
    def step(self, actions: torch.Tensor):
        """Step the physics of the environment."""

    @abc.abstractmethod
    def reset(self):
        """Reset the environment."""

    @abc.abstractmethod
    def reset_idx(self, env_ids: torch.Tensor):
        """Reset environments having the provided indices."""

    @property
    def observation_space(self):
        return self.obs_space

    @property
    def action_space(self):
        return self.act_space

    @property
    def num_envs(self) -> int:
        return self.num_environments

    @property
    def num_acts(self) -> int:
        return self.num_actions

    @property
    def num_obs(self) -> int:
        return self.num_observations


def mass_scale(sample: torch.Tensor, operation: str, base_mass: torch.Tensor) -> torch.Tensor:
    """Per-link mass scale the library applies for one DR mass sample
    ([N, L]): IsaacGym's 'scaling' sets m = m0 * s, 'additive' sets
    m = m0 + s, i.e. a scale of (m0 + s) / m0 (massless links keep scale 1)."""
    if operation == "scaling":
        return sample
    m0 = base_mass.to(sample.device, sample.dtype)
    safe = torch.where(m0 > 0, m0, torch.ones_like(m0))
    return torch.where(m0 > 0, (m0 + sample) / safe, torch.ones_like(sample))


class VecTask(Env):
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 24}
    #: sim.physx.contact_offset when the cfg has none: vec_task.py:442-482 sets
    #: no value, so IsaacGym's own 0.02 applies
    default_contact_offset = 0.02

    def __init__(self, config, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture: bool = False,
                 force_render: bool = False):
        self.cfg = config
        super().__init__(config, rl_device, sim_device, graphics_device_id, headless)
        self.virtual_screen_capture = virtual_screen_capture
        self.virtual_display = None
        self.force_render = force_render
        if not headless:
            warnings.warn("thormang_isaacgym_amd has no viewer; running headless")
        if self.cfg.get("physics_engine", "physx") not in ("physx", "flex"):
            raise ValueError(f"Invalid physics engine backend: {self.cfg['physics_engine']}")
        self.sim_params = self._parse_sim_params(self.cfg.get("physics_engine", "physx"), self.cfg["sim"])
        self.first_randomization = True
        self.original_props = {}
        self.dr_randomizations = {}
        self.actor_params_generator = None
        self.extern_actor_params = {}
        self.last_step = -1
        self.last_rand_step = -1
        self.frame_count = 0
        self.sim_initialized = False
        self.create_sim()
        self.sim_initialized = True
        self.viewer = None
        self.enable_viewer_sync = True
        self.allocate_buffers()
        self.obs_dict = {}

    # ------------------------------------------------------------ sim creation
    def _parse_sim_params(self, physics_engine: str, config_sim: Dict[str, Any]) -> Dict[str, Any]:
        if config_sim.get("up_axis", "z") not in ["z", "y"]:
            raise ValueError(f"Invalid physics up-axis: {config_sim['up_axis']}")
        if config_sim.get("up_axis", "z") != "z":
            raise ValueError("only up_axis 'z' is supported")
        out = dict(config_sim)
        out.setdefault("substeps", 2)
        out.setdefault("gravity", [0.0, 0.0, -9.81])
        return out

    def create_sim_object(self, model, asset_options: Dict[str, Any], env_spacing: float = 1.0):
        """gym.create_sim + load_asset + create_env/actor in one call (vec_task.py:279-295)."""
        from ...sim import Sim
        sp = abi.sim_params_from_cfg(self.sim_params, asset_options, self.num_envs, env_spacing,
                                     default_contact_offset=self.default_contact_offset)
        return Sim(model, sp, self.num_envs, self.device)

    def allocate_buffers(self):
        dev = self.device
        self.obs_buf = torch.zeros((self.num_envs, self.num_obs), device=dev, dtype=torch.float)
        self.states_buf = torch.zeros((self.num_envs, self.num_states), device=dev, dtype=torch.float)
        self.rew_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.float)
        self.reset_buf = torch.ones(self.num_envs, device=dev, dtype=torch.long)
        self.timeout_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.bool)
        self.progress_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.randomize_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.randomize_buf_bound = 0   # host-side upper bound of randomize_buf (see apply_randomizations)
        self.extras = {}

    def set_viewer(self):
        self.viewer = None

    def get_state(self):
        return torch.clamp(self.states_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)

    @abc.abstractmethod
    def pre_physics_step(self, actions: torch.Tensor):
        """Apply the actions to the environment."""

    @abc.abstractmethod
    def post_physics_step(self):
        """Compute reward and observations, reset any environments that require it."""

    def simulate(self):
        self.sim.simulate()
        self.frame_count += 1

    def step(self, actions: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor, Dict[str, Any]]:
        if self.dr_randomizations.get("actions", None):
            actions = self.dr_randomizations["actions"]["noise_lambda"](actions)
        action_tensor = torch.clamp(actions, -self.clip_actions, self.clip_actions)
        self.pre_physics_step(action_tensor)
        for _ in range(self.control_freq_inv):
            self.simulate()
        self.post_physics_step()
        self.timeout_buf = (self.progress_buf >= self.max_episode_length - 1) & (self.reset_buf != 0)
        if self.dr_randomizations.get("observations", None):
            self.obs_buf = self.dr_randomizations["observations"]["noise_lambda"](self.obs_buf)
        self.extras["time_outs"] = self.timeout_buf.to(self.rl_device)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    def _rl_out(self):
        """The step's return tuple on rl_device: the live buffers when rl_device
        is the sim GPU (no copy), copies when it is not (the CPU pipeline)."""
        if torch.device(self.rl_device) == torch.device(self.device):
            return self.obs_dict, self.rew_buf, self.reset_buf, self.extras
        obs = {k: v.to(self.rl_device) for k, v in self.obs_dict.items()}
        extras = dict(self.extras)
        extras["time_outs"] = self.extras["time_outs"].to(self.rl_device)
        return obs, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), extras

    def zero_actions(self) -> torch.Tensor:
        return torch.zeros([self.num_envs, self.num_actions], dtype=torch.float32, device=self.rl_device)

    def reset_idx(self, env_idx):
        pass

    def reset(self):
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict

    def reset_done(self):
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, done_env_ids

    def render(self, mode="rgb_array"):
        return None

    # ------------------------------------------------------------ domain randomisation
    @staticmethod
    def _sched(params, step):
        sched = params.get("schedule", None)
        steps = params.get("schedule_steps", None)
        if sched == "linear":
            return 1.0 / steps * min(step, steps)
        if sched == "constant":
            return 0.0 if step < steps else 1.0
        return 1.0

    def _sample(self, params, shape, step, gen=None, device=None):
        """generate_random_samples semantics: uniform / loguniform / gaussian, with schedule."""
        device = self.device if device is None else device
        dist = params["distribution"]
        lo, hi = params["range"]
        op = params.get("operation", "additive")
        s = self._sched(params, step)
        if dist == "gaussian":
            mu, var = lo, hi
            if op == "additive":
                mu, var = mu * s, var * s
            elif op == "scaling":
                var = var * s
                mu = mu * s + 1.0 * (1.0 - s)
            x = torch.randn(shape, device=device, generator=gen) * var + mu
        elif dist in ("uniform", "loguniform"):
            if op == "additive":
                lo, hi = lo * s, hi * s
            elif op == "scaling":
                lo, hi = lo * s + 1.0 * (1.0 - s), hi * s + 1.0 * (1.0 - s)
            u = torch.rand(shape, device=device, generator=gen)
            if dist == "loguniform":
                x = torch.exp(math.log(lo) + u * (math.log(hi) - math.log(lo)))
            else:
                x = lo + u * (hi - lo)
        else:
            raise ValueError(f"unknown distribution {dist}")
        return x

    def _base_link_mass(self) -> torch.Tensor:
        """[L] URDF link masses of the sim's model (the DR reference masses)."""
        return torch.as_tensor(self.sim.desc.arrays["link_inertia"][:, 0], device=self.device)

    def apply_randomizations(self, dr_params):
        rand_freq = dr_params.get("frequency", 1)
        self.last_step = self.frame_count
        if self.first_randomization:
            do_nonenv = True
            env_ids = torch.arange(self.num_envs, device=self.device)
        else:
            do_nonenv = (self.last_step - self.last_rand_step) >= rand_freq
            # vec_task.py:559-563.  Nothing on the reference's path increments
            # randomize_buf, so per-env re-sampling never fires there; a task that
            # does increment it raises self.randomize_buf_bound (host-side upper
            # bound), which keeps the usual path free of a device sync.
            if self.randomize_buf_bound >= rand_freq:
                rand_envs = (self.randomize_buf >= rand_freq) & (self.reset_buf != 0)
                env_ids = torch.nonzero(rand_envs, as_tuple=False).squeeze(-1)
                self.randomize_buf[rand_envs] = 0
            else:
                env_ids = torch.zeros(0, dtype=torch.long, device=self.device)
        if do_nonenv:
            self.last_rand_step = self.last_step
        for nonphysical in ("observations", "actions"):
            if nonphysical in dr_params and do_nonenv:
                p = dr_params[nonphysical]
                op = operator.add if p["operation"] == "additive" else operator.mul
                s = self._sched(p, self.last_step)
                if p["distribution"] == "gaussian":
                    mu, var = p["range"]
                    mu_c, var_c = p.get("range_correlated", [0.0, 0.0])
                    if p["operation"] == "additive":
                        mu, var, mu_c, var_c = mu * s, var * s, mu_c * s, var_c * s
                    else:
                        var, mu = var * s, mu * s + 1.0 * (1.0 - s)
                        var_c, mu_c = var_c * s, mu_c * s + 1.0 * (1.0 - s)

                    def noise_lambda(tensor, name=nonphysical, op=op):
                        q = self.dr_randomizations[name]
                        corr = q.get("corr", None)
                        if corr is None:
                            corr = torch.randn_like(tensor)
                            q["corr"] = corr
                        corr = corr * q["var_corr"] + q["mu_corr"]
                        return op(tensor, corr + torch.randn_like(tensor) * q["var"] + q["mu"])

                    self.dr_randomizations[nonphysical] = {"mu": mu, "var": var, "mu_corr": mu_c, "var_corr": var_c,
                                                           "noise_lambda": noise_lambda}
                else:
                    lo, hi = p["range"]
                    lo_c, hi_c = p.get("range_correlated", [0.0, 0.0])
                    if p["operation"] == "additive":
                        lo, hi, lo_c, hi_c = lo * s, hi * s, lo_c * s, hi_c * s
                    else:
                        lo, hi = lo * s + 1.0 * (1.0 - s), hi * s + 1.0 * (1.0 - s)
                        lo_c, hi_c = lo_c * s + 1.0 * (1.0 - s), hi_c * s + 1.0 * (1.0 - s)

                    def noise_lambda(tensor, name=nonphysical, op=op):
                        q = self.dr_randomizations[name]
                        corr = q.get("corr", None)
                        if corr is None:
                            corr = torch.randn_like(tensor)
                            q["corr"] = corr
                        corr = corr * (q["hi_corr"] - q["lo_corr"]) + q["lo_corr"]
                        return op(tensor, corr + torch.rand_like(tensor) * (q["hi"] - q["lo"]) + q["lo"])

                    self.dr_randomizations[nonphysical] = {"lo": lo, "hi": hi, "lo_corr": lo_c, "hi_corr": hi_c,
                                                           "noise_lambda": noise_lambda}
        if "sim_params" in dr_params and do_nonenv:
            for attr, p in dr_params["sim_params"].items():
                if attr != "gravity":
                    continue
                # three numbers drawn on the host (as dr_utils does with numpy):
                # no device round trip on this periodic path
                base = torch.tensor(self.sim_params["gravity"], dtype=torch.float32)
                smp = self._sample(p, (3,), self.last_step, device="cpu")
                g = base * smp if p.get("operation", "additive") == "scaling" else base + smp
                self.sim.set_gravity(g.tolist())
        n = int(env_ids.numel())
        if n > 0:
            for actor, props in dr_params.get("actor_params", {}).items():
                rb = props.get("rigid_body_properties", {})
                if "mass" in rb:
                    p = rb["mass"]
                    if (p.get("setup_only", False) and not self.sim_initialized) or not p.get("setup_only", False):
                        smp = self._sample(p, (self.num_envs, self.sim.L), self.last_step)
                        scale = mass_scale(smp, p.get("operation", "additive"), self._base_link_mass())
                        self.sim.set_body_mass_scale_indexed(scale.contiguous(), env_ids)
                rs = props.get("rigid_shape_properties", {})
                if "friction" in rs and self.sim.S > 0:
                    p = rs["friction"]
                    base = torch.as_tensor(self.sim.desc.arrays["shape_friction"], device=self.device)
                    smp = self._sample(p, (self.num_envs, self.sim.S), self.last_step)
                    mu = base * smp if p.get("operation", "additive") == "scaling" else base + smp
                    self.sim.set_shape_friction_indexed(mu.contiguous(), env_ids)
        self.first_randomization = False

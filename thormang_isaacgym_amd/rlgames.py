"""rl_games adaptor: the caller side of the hot path.

The reference trains through ``train.py`` -> rl_games ``Runner`` -> the
``'RLGPU'`` vec-env, which wraps ``isaacgymenvs.make`` (train.py:99-131,
export.py:80-103; the adaptor class itself lives in IsaacGymEnvs'
``utils/rlgames_utils.py``, not vendored in the reference).  This module
provides the same pieces over this package's tasks:

* ``get_rlgames_env_creator`` -- the ``create_env_thunk`` of train.py:99-122;
* ``RLGPUEnv`` -- the vec-env rl_games drives: ``step`` / ``reset`` /
  ``reset_done`` / ``get_number_of_agents`` / ``get_env_info`` (+ the
  set_train_info / env-state hooks), tensors stay on the env's GPU;
* ``EpisodeStats`` -- per-env episode return / length accumulation on the
  device and the per-iteration all-rank gather of their sums;
* ``register`` -- registers both with rl_games' ``vecenv`` /
  ``env_configurations`` when rl_games is importable (it is not in this image);
* ``PolicyExport`` / ``export_policy`` -- export.py:130-170: the trained model
  wrapped to return ``clamp(mu, -1, 1)`` and traced with torch.jit; ONNX is
  written when the ``onnx`` package is present (it is not in this image) and
  the traced TorchScript module is the portable artefact otherwise.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict

import torch

#: stand-in for rl_games.common.env_configurations.configurations when rl_games is absent
configurations: Dict[str, Dict[str, Any]] = {}


def get_rlgames_env_creator(seed: int, task_config: dict, task_name: str, sim_device: str, rl_device: str,
                            graphics_device_id: int = -1, headless: bool = True, multi_gpu: bool = False,
                            virtual_screen_capture: bool = False, force_render: bool = False,
                            post_create_hook: Callable | None = None) -> Callable:
    """train.py:99-122: a thunk creating the task env (torchrun rank -> device)."""
    def create_env(**kwargs):
        from . import make
        dev_sim, dev_rl = sim_device, rl_device
        if multi_gpu:
            # one process per GPU (torchrun): LOCAL_RANK -> device.  The seed is
            # taken as given: the caller (train.py:80, cfg.seed += LOCAL_RANK)
            # has already made it distinct per rank, and it keys the in-kernel
            # Philox streams
            local = int(os.getenv("LOCAL_RANK", "0"))
            dev_sim = dev_rl = f"cuda:{local}"
        env = make(seed=seed, task=task_name, num_envs=task_config["env"]["numEnvs"], sim_device=dev_sim,
                   rl_device=dev_rl, graphics_device_id=graphics_device_id, headless=headless,
                   virtual_screen_capture=virtual_screen_capture, force_render=force_render, cfg=task_config)
        if post_create_hook is not None:
            post_create_hook()
        return env
    return create_env


class EpisodeStats:
    """Per-iteration host gather of episode returns and lengths (north_star: the
    env batch shards across GPUs with no collective on the hot path, "only a
    per-iteration host gather of returns").

    ``update(rew, reset)`` runs after every ``env.step`` on the env's device
    with no host synchronisation: it accumulates each env's running return and
    length and folds finished episodes (``reset != 0``) into three device sums.
    ``gather()`` -- once per PPO iteration -- sums those over all ranks (one
    all-reduce of 3 float64 scalars when torch.distributed is initialised;
    gloo reduces on the host, RCCL on the device), resets the sums and returns
    the job-wide ``{"episodes", "mean_return", "mean_length"}`` on every rank."""

    def __init__(self, num_envs: int, device):
        self.device = torch.device(device)
        self.ret = torch.zeros(num_envs, dtype=torch.float64, device=self.device)
        self.len = torch.zeros(num_envs, dtype=torch.float64, device=self.device)
        self.sums = torch.zeros(3, dtype=torch.float64, device=self.device)   # return, length, episodes

    def update(self, rew: torch.Tensor, reset: torch.Tensor) -> None:
        self.ret += rew.to(torch.float64)
        self.len += 1.0
        done = reset != 0
        d = done.to(torch.float64)
        self.sums += torch.stack([(self.ret * d).sum(), (self.len * d).sum(), d.sum()])
        self.ret.masked_fill_(done, 0.0)
        self.len.masked_fill_(done, 0.0)

    def gather(self) -> dict:
        import torch.distributed as dist
        t = self.sums.clone()
        if dist.is_available() and dist.is_initialized():
            if dist.get_backend() == "gloo":
                t = t.cpu()
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        ret, length, n = (float(x) for x in t.cpu())
        self.sums.zero_()
        return {"episodes": int(round(n)), "mean_return": ret / n if n > 0 else float("nan"),
                "mean_length": length / n if n > 0 else float("nan")}


class RLGPUEnv:
    """rl_games ``IVecEnv`` over a task env: the env stays on its GPU and the
    tensors pass through unchanged (obs dict, reward, done, extras)."""

    def __init__(self, config_name: str, num_actors: int, **kwargs):
        conf = _configurations().get(config_name)
        if conf is None:
            raise KeyError(f"env configuration {config_name!r} is not registered")
        self.env = conf["env_creator"](**kwargs)

    def step(self, actions):
        return self.env.step(actions)

    def reset(self):
        return self.env.reset()

    def reset_done(self):
        return self.env.reset_done()

    def get_number_of_agents(self) -> int:
        f = getattr(self.env, "get_number_of_agents", None)   # VecTask has none: one agent per env
        return f() if f is not None else 1

    def get_env_info(self) -> dict:
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space}
        if hasattr(self.env, "amp_observation_space"):
            info["amp_observation_space"] = self.env.amp_observation_space
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info

    def set_train_info(self, env_frames, *args, **kwargs):
        if hasattr(self.env, "set_train_info"):
            self.env.set_train_info(env_frames, *args, **kwargs)

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass


def _configurations() -> Dict[str, Dict[str, Any]]:
    try:
        from rl_games.common import env_configurations
        return env_configurations.configurations
    except ImportError:
        return configurations


def register(create_env: Callable, name: str = "rlgpu") -> None:
    """train.py:125-131: register the 'RLGPU' vec-env and the env configuration."""
    conf = {"vecenv_type": "RLGPU", "env_creator": create_env}
    try:
        from rl_games.common import env_configurations, vecenv
        vecenv.register("RLGPU", lambda config_name, num_actors, **kw: RLGPUEnv(config_name, num_actors, **kw))
        env_configurations.register(name, conf)
    except ImportError:
        configurations[name] = conf


class PolicyExport(torch.nn.Module):
    """export.py:133-155 ModelWrapper: deterministic action = clamp(mu, -1, 1).
    ``model`` is an rl_games-style module taking the input dict and returning
    ``{'mus': ...}``, or any callable obs -> mu."""

    def __init__(self, model):
        super().__init__()
        self._model = model

    def forward(self, obs):
        out = self._model({"is_train": False, "prev_actions": None, "obs": obs, "rnn_states": None}) \
            if getattr(self._model, "takes_input_dict", False) else self._model(obs)
        mu = out["mus"] if isinstance(out, dict) else out
        return torch.clamp(mu, -1.0, 1.0)


def export_policy(model, obs_dim: int, path: str, device: str = "cpu") -> str:
    """Trace the wrapped policy (export.py:158-166) and write it.  Writes ONNX
    (input 'obs', output 'actions') when the onnx package is importable,
    else TorchScript; returns the path written."""
    inputs = torch.zeros((1, obs_dim), device=device)
    with torch.no_grad():
        traced = torch.jit.trace(PolicyExport(model).to(device), (inputs,), check_trace=False)
    try:
        import onnx  # noqa: F401
        out = os.path.splitext(path)[0] + ".onnx"
        torch.onnx.export(traced, (inputs,), out, input_names=["obs"], output_names=["actions"])
    except ImportError:
        out = os.path.splitext(path)[0] + ".pt"
        traced.save(out)
    return out

"""Task configs with the reference's schema (isaacgymenvs/cfg/task/*.yaml).

``load_task_cfg`` returns the plain dict ``isaacgymenvs.make`` builds with
``omegaconf_to_dict(cfg.task)`` (isaacgymenvs/__init__.py:35-41), resolving the
Hydra interpolations the reference uses (cfg/config.yaml: physics_engine,
pipeline -> sim.use_gpu_pipeline, sim_device -> physx.use_gpu, num_threads,
num_subscenes)."""
from __future__ import annotations

import copy
import os

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))


def load_task_cfg(task: str = "Gogoro", num_envs: int | None = None, sim_device: str = "cuda:0",
                  pipeline: str = "gpu", physics_engine: str = "physx", num_threads: int = 4,
                  num_subscenes: int = 4, overrides: dict | None = None) -> dict:
    path = os.path.join(HERE, "task", f"{task}.yaml")
    if not os.path.exists(path):
        raise KeyError(f"no task config {task!r} (have: {sorted(f[:-5] for f in os.listdir(os.path.join(HERE, 'task')))})")
    with open(path) as f:
        cfg = yaml.safe_load(f)
    cfg["physics_engine"] = physics_engine
    cfg["sim"]["use_gpu_pipeline"] = pipeline.lower() == "gpu"
    px = cfg["sim"].setdefault("physx", {})
    px["use_gpu"] = "cuda" in sim_device.lower()
    px["num_threads"] = num_threads
    px["num_subscenes"] = num_subscenes
    if num_envs is not None:
        cfg["env"]["numEnvs"] = int(num_envs)
    for k, v in (overrides or {}).items():
        _set(cfg, k, v)
    return cfg


def _set(cfg, dotted, value):
    keys = dotted.split(".")
    d = cfg
    for k in keys[:-1]:
        d = d.setdefault(k, {})
    d[keys[-1]] = copy.deepcopy(value)

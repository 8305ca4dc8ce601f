"""MI355X-native vectorised RL environment for the Gogoro scooter and Thormang3
humanoid tasks, behind the IsaacGymEnvs ``VecTask`` API (drop-in for
Yougo-robotics/thormang_isaacgym's task path).

``make`` mirrors ``isaacgymenvs.make`` (isaacgymenvs/__init__.py:14-55) minus
Hydra: it builds the task dict from our cfg/ (or takes a ready dict) and
returns the task object (the reference wraps it in rl_games' RLGPUEnv)."""
from __future__ import annotations

__version__ = "0.1.0"


def make(seed: int, task: str, num_envs: int, sim_device: str, rl_device: str, graphics_device_id: int = -1,
         headless: bool = True, multi_gpu: bool = False, virtual_screen_capture: bool = False,
         force_render: bool = False, cfg: dict | None = None):
    import torch

    from .cfg import load_task_cfg
    from .tasks import isaacgym_task_map
    if cfg is None:
        cfg = load_task_cfg(task, num_envs=num_envs, sim_device=sim_device)
    cfg = dict(cfg)
    cfg["seed"] = seed
    torch.manual_seed(seed)
    return isaacgym_task_map[cfg["name"]](cfg=cfg, rl_device=rl_device, sim_device=sim_device,
                                          graphics_device_id=graphics_device_id, headless=headless,
                                          virtual_screen_capture=virtual_screen_capture, force_render=force_render)

"""rl_games adaptor (thormang_isaacgym_amd/rlgames.py): registration, the
vec-env protocol over a task env, and the policy export path of export.py."""
import os

import pytest
import torch

from thormang_isaacgym_amd import rlgames


class _FakeEnv:
    num_states = 0
    action_space = "A"
    observation_space = "O"

    def __init__(self):
        self.calls = []

    def step(self, a):
        self.calls.append("step")
        return {"obs": a * 2}, a.sum(1), torch.zeros(a.shape[0], dtype=torch.long), {"time_outs": None}

    def reset(self):
        self.calls.append("reset")
        return {"obs": torch.zeros(2, 3)}

    def reset_done(self):
        return {"obs": torch.zeros(2, 3)}, torch.zeros(0, dtype=torch.long)


def test_register_and_drive_vecenv():
    made = []
    rlgames.register(lambda **kw: made.append(_FakeEnv()) or made[-1], name="rlgpu_test")
    env = rlgames.RLGPUEnv("rlgpu_test", 2)
    assert env.get_env_info() == {"action_space": "A", "observation_space": "O"}
    assert env.get_number_of_agents() == 1
    obs, rew, done, info = env.step(torch.ones(2, 3))
    assert torch.equal(obs["obs"], 2 * torch.ones(2, 3)) and rew.tolist() == [3.0, 3.0]
    env.reset()
    assert made[0].calls == ["step", "reset"]
    with pytest.raises(KeyError):
        rlgames.RLGPUEnv("not_registered", 1)


def test_export_policy_clamps_and_round_trips(tmp_path):
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.ELU(), torch.nn.Linear(16, 1))
    with torch.no_grad():
        net[2].bias.fill_(3.0)                   # mu far outside [-1, 1]
    out = rlgames.export_policy(net, 6, str(tmp_path / "policy"))
    assert os.path.exists(out)
    if out.endswith(".pt"):
        m = torch.jit.load(out)
        x = torch.rand(4, 6) * 2 - 1
        y = m(x)
        assert y.shape == (4, 1) and float(y.max()) <= 1.0
        torch.testing.assert_close(y, torch.clamp(net(x), -1, 1))


@pytest.mark.gpu
def test_rlgpu_env_over_gogoro_paper_on_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg("GogoroPaper", num_envs=256)
    rlgames.register(rlgames.get_rlgames_env_creator(7, cfg, "GogoroPaper", "cuda:0", "cuda:0"), name="rlgpu_paper")
    env = rlgames.RLGPUEnv("rlgpu_paper", 256)
    info = env.get_env_info()
    assert info["observation_space"].shape == (160,) and info["action_space"].shape == (1,)
    obs = env.reset()["obs"]
    assert obs.shape == (256, 160) and obs.device.type == "cuda"
    policy = torch.jit.trace(rlgames.PolicyExport(torch.nn.Linear(160, 1).cuda()), (obs,))
    for _ in range(20):
        obs, rew, done, extras = env.step(policy(obs))
        obs = obs["obs"]
    assert torch.isfinite(obs).all() and rew.shape == (256,) and done.dtype == torch.long

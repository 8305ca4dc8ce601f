"""Developer probe: GogoroPaper step at 4096 envs in three variants (fused
step; separate calls; pushes off) so a rocprofv3 kernel trace shows what the
compose launch costs in each.  Variant by argv[1]: fused | unfused | nopush."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import thormang_isaacgym_amd as tia  # noqa: E402
from thormang_isaacgym_amd.tasks import gogoro_paper as gp  # noqa: E402

v = sys.argv[1]
if v == "unfused":
    os.environ["TG_PAPER_UNFUSED"] = "1"
if v == "nopush":
    gp.PUSH_ROBOT = False
env = tia.make(seed=1, task="GogoroPaper", num_envs=4096, sim_device="cuda:0", rl_device="cuda:0")
g = torch.Generator(device="cuda:0").manual_seed(2)
for _ in range(200):
    env.step(torch.rand(4096, 1, device="cuda:0", generator=g) * 2 - 1)
torch.cuda.synchronize()
print(v, "ok")

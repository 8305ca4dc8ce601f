"""Developer check (GPU, TG_CH8_DBG=2 build): how often the impulse top-down
pass's register-forwarded parent responses differ bitwise from the values
the parent stored (first mismatch: step, group, lane)."""
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
import thormang_isaacgym_amd as tia  # noqa: E402
from thormang_isaacgym_amd._lib import lib  # noqa: E402

env = tia.make(seed=3, task="ThormangWalk", num_envs=256, sim_device="cuda:0", rl_device="cuda:0")
g = torch.Generator(device="cuda:0").manual_seed(9)
for _ in range(3):
    env.step(torch.rand(256, 33, device="cuda:0", generator=g) * 2 - 1)
torch.cuda.synchronize()
out = (C.c_uint * 8)()
lib().tg_ch8_read(out)
print("mismatches", out[0], "of", out[1], "first: step", int(out[2]) - 1, "group", out[3], "lane", out[4])

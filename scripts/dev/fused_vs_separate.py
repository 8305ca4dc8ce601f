"""Developer diagnostic: per-step max |fused - separate| of the Gogoro step
(obs, rew, root) under the env switches given on the command line."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import thormang_isaacgym_amd as tia
from thormang_isaacgym_amd.tasks.base.vec_task import VecTask
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    os.environ[k] = v
envs = [tia.make(seed=21, task="Gogoro", num_envs=512, sim_device="cuda:0", rl_device="cuda:0") for _ in range(2)]
f, u = envs
g = torch.Generator(device="cuda:0").manual_seed(9)
for t in range(40):
    a = torch.rand(512, 1, device="cuda:0", generator=g) * 2 - 1
    f.step(a)
    VecTask.step(u, a)
    torch.cuda.synchronize()
    same = torch.equal(f.reset_buf, u.reset_buf) and torch.equal(f.progress_buf, u.progress_buf)
    d = [float((x - y).abs().max()) for x, y in ((f.obs_buf, u.obs_buf), (f.rew_buf, u.rew_buf), (f.root_tensor, u.root_tensor))]
    print(t, same, "obs %.2e rew %.2e root %.2e" % tuple(d), "resets", int(f.reset_buf.sum()))

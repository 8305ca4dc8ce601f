"""Developer probe (GPU): is a task's step deterministic?  Two envs from the
same seed step the same actions side by side; any bitwise difference in
observations, rewards, resets or root / dof states is reported with its first
(step, env).

    python scripts/dev/determinism.py [task] [num_envs] [steps]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import thormang_isaacgym_amd as tia  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "Gogoro"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
envs = [tia.make(seed=5, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0") for _ in range(2)]
g = torch.Generator(device="cuda:0").manual_seed(7)
first = {}
count = {}
for t in range(steps):
    a = torch.rand(n, envs[0].num_actions, device="cuda:0", generator=g) * 2 - 1
    outs = [e.step(a) for e in envs]
    any_diff = False
    pairs = {"obs": (outs[0][0]["obs"], outs[1][0]["obs"]), "rew": (outs[0][1], outs[1][1]),
             "reset": (outs[0][2], outs[1][2]),
             "root": (envs[0].root_tensor, envs[1].root_tensor)}
    for k, (x, y) in pairs.items():
        d = (x != y)
        if d.dim() > 1:
            d = d.any(1)
        nd = int(d.sum())
        if nd:
            count[k] = count.get(k, 0) + nd
            if k not in first:
                first[k] = (t, int(torch.nonzero(d)[0]))
                dd = (x.float() - y.float()).abs().max()
                print(f"{task}: {k} differs first at step {t} env {first[k][1]} (max |d| {float(dd):.3e})", flush=True)
            any_diff = True
    if any_diff:   # re-sync every shared buffer, so that one difference does not propagate
        for k, x in envs[0]._buf_tensors.items():
            if x is not None and envs[1]._buf_tensors.get(k) is not None:
                envs[1]._buf_tensors[k].copy_(x)
print(task, n, steps, "differing env-steps per buffer:", count or "none")

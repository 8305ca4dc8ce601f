"""Developer probe (GPU): the per-step states of a fixed ThormangWalk run
under the library TG_LIB_PATH points at (first K steps), saved to OUT.npz; with
two files given, reports the first step and field at which they differ and by
how much (a rounding-level first difference that grows is arithmetic, a large
first difference is a semantic change).

    TG_LIB_PATH=a.so python scripts/dev/step_states.py run out_a.npz [task] [steps]
    python scripts/dev/step_states.py cmp out_a.npz out_b.npz
"""
import sys

import numpy as np

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    T = int(a["steps"])
    for t in range(T):
        for k in ("root", "dof", "obs", "rew"):
            x, y = a[f"{k}{t}"], b[f"{k}{t}"]
            if not np.array_equal(x, y):
                d = np.abs(x.astype(np.float64) - y.astype(np.float64))
                i = np.unravel_index(int(np.argmax(d)), d.shape)
                print(f"step {t}: {k} differs, max |d| {d.max():.3e} at {i}, {int((d > 0).sum())} entries")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, ".")
import thormang_isaacgym_amd as tia  # noqa: E402

task = sys.argv[3] if len(sys.argv) > 3 else "ThormangWalk"
T = int(sys.argv[4]) if len(sys.argv) > 4 else 12
n = 256
env = tia.make(seed=3, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
g = torch.Generator(device="cuda:0").manual_seed(9)
out = {"steps": T}
for t in range(T):
    obs, rew, reset, extras = env.step(torch.rand(n, env.num_actions, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    out[f"root{t}"] = env.sim.root_state.cpu().numpy()
    out[f"dof{t}"] = env.sim.dof_state.cpu().numpy()
    out[f"obs{t}"] = obs["obs"].cpu().numpy()
    out[f"rew{t}"] = rew.cpu().numpy()
np.savez(sys.argv[2], **out)

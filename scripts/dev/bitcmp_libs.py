"""Developer probe (GPU): the final state of a fixed run of each task under the
library TG_LIB_PATH points at, saved to OUT.npz; with two files given,
compares them bit for bit (library builds that should differ only in
instruction scheduling must agree exactly).

    TG_LIB_PATH=a.so python scripts/dev/bitcmp_libs.py run out_a.npz
    python scripts/dev/bitcmp_libs.py cmp out_a.npz out_b.npz
"""
import sys

import numpy as np

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = 0
    for k in sorted(a.files):
        same = np.array_equal(a[k], b[k], equal_nan=True)
        d = float(np.nanmax(np.abs(a[k].astype(np.float64) - b[k].astype(np.float64)))) if a[k].size else 0.0
        print(f"{k:28s} {'identical' if same else 'DIFFERENT'} max|d| {d:.3e}")
        bad += not same
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

sys.path.insert(0, ".")
import thormang_isaacgym_amd as tia  # noqa: E402

from thormang_isaacgym_amd.cfg import load_task_cfg  # noqa: E402

out = {}
for task, n, na in (("ThormangWalk", 1024, 33), ("ThormangWalkDR", 1024, 33), ("Gogoro", 1024, 1),
                    ("GogoroPaper", 1024, 1), ("ThormangWalk+wb", 1024, 33)):
    name, _, var = task.partition("+")
    cfg = load_task_cfg(name, num_envs=n)
    if var == "wb":   # the whole-body contact model (thormang_wb)
        cfg["env"]["asset"] = dict(cfg["env"].get("asset", {}), wholeBodyCollision=True)
    env = tia.make(seed=3, task=name, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
    g = torch.Generator(device="cuda:0").manual_seed(9)
    for _ in range(100):
        obs, rew, reset, extras = env.step(torch.rand(n, na, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    out[f"{task}_obs"] = obs["obs"].cpu().numpy()
    out[f"{task}_rew"] = rew.cpu().numpy()
    out[f"{task}_root"] = env.sim.root_state.cpu().numpy()
    out[f"{task}_dof"] = env.sim.dof_state.cpu().numpy()
    del env
np.savez(sys.argv[2], **out)
print("saved", sys.argv[2])

"""Developer diagnostic: free-running Gogoro-on-terrain GPU vs oracle, the
per-step max |obs| error and the env that holds it (drift vs event jumps)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests import gpu_harness as H  # noqa: E402
from tests.oracle_lib import set_heightfield  # noqa: E402
from thormang_isaacgym_amd.tasks import gogoro as gmod  # noqa: E402

n, steps, seed = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 60, 6
torch.manual_seed(5)
saved, gmod.USE_TERAIN = gmod.USE_TERAIN, True
env = H.make_gpu_gogoro(H.parity_cfg(n, max_steps=300), H.NumpyDraws(seed))
gmod.USE_TERAIN = saved
t = env.terrain
o = -float(env._terrain_start_mid)
set_heightfield(t.heightsamples.cpu().numpy(), t.V_scale, t.H_scale, o, o, friction=0.98)
orc = H.OracleGogoro(H.parity_cfg(n, max_steps=300), H.NumpyDraws(seed), spawn_z=env.root_reset_tensor[:, 2].cpu().numpy())
obs = orc.a["obs_buf"].copy()
for k in range(steps):
    act = H.balance_policy(obs)
    od, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    oo, orw, ore, _ = orc.step(act[:, 0])
    e = np.abs(od["obs"].cpu().numpy() - oo)
    er = np.abs(env.root_tensor.cpu().numpy() - orc.a["root"])
    i = int(e.max(1).argmax())
    print(f"step {k:3d} obs {e.max():.2e} env {i:2d} comp {int(e[i].argmax())} root {er.max():.2e} "
          f"reset {int(reset.sum())}/{int(ore.sum())}")
    obs = oo.copy()
set_heightfield(None)

# teacher-forced along the same start: the oracle re-synced from the GPU state
# before every step (one-step errors; actions from the GPU observations)
if len(sys.argv) > 2:
    torch.manual_seed(5)
    gmod.USE_TERAIN = True
    env = H.make_gpu_gogoro(H.parity_cfg(n, max_steps=300), H.NumpyDraws(seed))
    gmod.USE_TERAIN = saved
    set_heightfield(t.heightsamples.cpu().numpy(), t.V_scale, t.H_scale, o, o, friction=0.98)
    orc = H.OracleGogoro(H.parity_cfg(n, max_steps=300), H.NumpyDraws(seed), spawn_z=env.root_reset_tensor[:, 2].cpu().numpy())
    obs = orc.a["obs_buf"].copy()
    for k in range(steps):
        H.sync_oracle_from_gpu(orc, env)
        act = H.balance_policy(obs)
        od = env.step(torch.from_numpy(act).to("cuda:0"))[0]["obs"].cpu().numpy()
        oo = orc.step(act[:, 0])[0]
        e = np.abs(od - oo)
        i = int(e.max(1).argmax())
        print(f"forced step {k:3d} obs {e.max():.2e} env {i:2d} comp {int(e[i].argmax())}")
        obs = od
    set_heightfield(None)

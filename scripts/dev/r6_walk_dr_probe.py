"""Developer probe (GPU): the 16384-env teacher-forced ThormangWalkDR run of
test_gpu_walk_dr_16384_envs (seed 12, DR live, 100 steps) -- per step the
worst env's obs / root error against the fp64 oracle, and for the worst
env-steps the env's state (pelvis height, its mass scale range, contact), so a
rare per-env discrepancy can be located.  TG_LIB_PATH selects the library.

    python scripts/dev/r6_walk_dr_probe.py [num_envs] [steps] [dr 0/1]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.gpu_harness import (NumpyDraws, OracleWalk, make_gpu_walk, sync_dr, sync_oracle_from_gpu,  # noqa: E402
                               walk_cfg)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dr = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
tseed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
seed = 12
mk = lambda: walk_cfg(n, "ThormangWalkDR", dr=dr)
env = make_gpu_walk(mk(), NumpyDraws(seed), torch_seed=tseed)
orc = OracleWalk(mk(), NumpyDraws(seed))
ctl = OracleWalk(mk(), NumpyDraws(seed), precision="f32")
rs = np.random.default_rng(seed + 100)
rows = []
for t in range(steps):
    for o in (orc, ctl):
        sync_oracle_from_gpu(o, env)
        sync_dr(o, env)
    pre_root = env.root_tensor.cpu().numpy().copy()
    act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
    od, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
    o_obs, o_rew, o_reset, _ = orc.step(act)
    ctl.step(act)
    c_root = ctl.a["root"].copy()
    g_obs = od["obs"].cpu().numpy()
    e = np.abs(g_obs - o_obs).max(1)
    er = np.abs(env.root_tensor.cpu().numpy() - orc.a["root"]).max(1)
    ec = np.abs(c_root - orc.a["root"]).max(1)
    i = int(np.argmax(er))
    rows.append((float(er[i]), float(ec[i]), float(ec.max()), float(e[i]), t, i, float(pre_root[i, 2]),
                 int(np.sum(er > 1e-3)), int(np.sum(ec > 1e-3))))
rows.sort(reverse=True)
lib = os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so"))
print(f"== {lib} n {n} dr {dr} torch seed {tseed}: worst GPU root err (fp32 control's at that env, its worst), obs err, "
      "step, env, pelvis z before, envs over 1e-3 that step (GPU, control)")
for r in rows[:6]:
    print("  root %.2e (ctl %.2e, ctl max %.2e) obs %.2e step %3d env %5d z %.3f bad %d/%d" % r, flush=True)

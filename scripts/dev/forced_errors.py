"""Teacher-forced GPU-vs-oracle one-step errors for the current libtgsim
(TG_LIB_PATH selects a developer build): ThormangWalk at N envs, and the
fp32 oracle's own one-step error against the fp64 oracle on the same states
for scale.  Prints one JSON line.  Developer tool for the drift study.

    TG_LIB_PATH=... python scripts/dev/forced_errors.py [--envs 8192] [--steps 100] [--label X]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--label", default=os.path.basename(os.environ.get("TG_LIB_PATH", "libtgsim.so")))
    a = ap.parse_args()
    import torch
    from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_oracle_from_gpu, walk_cfg
    n = a.envs
    env = make_gpu_walk(walk_cfg(n), NumpyDraws(a.seed))
    orc = OracleWalk(walk_cfg(n), NumpyDraws(a.seed))
    rs = np.random.default_rng(a.seed + 100)
    e_obs, e_rew = [], []
    worst = (0.0, -1, -1)
    for t in range(a.steps):
        sync_oracle_from_gpu(orc, env)
        act = rs.uniform(-0.5, 0.5, (n, orc.D)).astype(np.float32)
        od, rew, _, _ = env.step(torch.from_numpy(act).to("cuda:0"))
        o_obs, o_rew, _, _ = orc.step(act)
        eo = np.abs(od["obs"].cpu().numpy() - o_obs).max(axis=1)
        er = np.abs(rew.cpu().numpy() - o_rew)
        e_obs.append(eo)
        e_rew.append(er)
        if er.max() > worst[0]:
            worst = (float(er.max()), t, int(er.argmax()))
    eo, er = np.concatenate(e_obs), np.concatenate(e_rew)
    print(json.dumps({"label": a.label, "envs": n, "steps": a.steps, "obs_max": float(eo.max()),
                      "obs_p999": float(np.quantile(eo, 0.999)), "obs_median": float(np.median(eo)),
                      "rew_max": float(er.max()), "rew_p999": float(np.quantile(er, 0.999)),
                      "rew_median": float(np.median(er)), "worst_rew": worst}), flush=True)


if __name__ == "__main__":
    main()

"""Free-running divergence study: is the GPU-vs-oracle drift chaos or model mismatch?

    python scripts/parity_drift.py WORKLOAD [--steps 1000] [--envs N] [--no-gpu] [--out DIR]

WORKLOAD: gogoro (free base, balance policy), gogoro_random (free base, the
bench's U(-1,1) actions), gogoro_fixbase (DEBUGFIXBASE),
walk (random actions), walk_stand (zero actions), walk_fixbase.

One reference run -- the fp64 oracle env (oracle/physics_ref.c + the task
oracle) -- chooses every action; three other runs replay exactly those actions
and are compared with it step by step:

  gpu        the product env on the MI355X (fp32 HIP kernels)
  perturbed  the fp64 oracle, initial root position and joint positions
             shifted by 1e-6 (random signs)
  f32        the same oracle compiled with real = float (liboracle_f32.so)

``--variants label=lib.so,...`` adds one GPU column per developer build of
libtgsim (each run in its own process with TG_LIB_PATH; e.g. a build with
-DTG_PRECISE_SINCOS or -fno-fast-math), to locate a GPU-specific drift.

Per step: max and median over envs of |obs - obs_ref| and the number of envs
whose reset flags have differed so far.  The "horizon" of a run is the first
step whose max error exceeds 1e-3 (north_star tolerance).  If the GPU run's
horizon matches the perturbed and fp32 runs' horizons, the divergence is the
task's sensitivity to 1e-6-size differences (chaos), not a modelling
difference.  Writes <out>/drift_<workload>.json and a text table; the copies
judged are committed under profiles/.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tests.gpu_harness import (NumpyDraws, OracleGogoro, OracleWalk, balance_policy, make_gpu_gogoro,  # noqa: E402
                               make_gpu_walk, parity_cfg, walk_cfg)

TOL = 1e-3


def _walk_cfg(n, fix_base):
    # fixed base: the pelvis hangs 0.5 m higher, so the feet swing free of the ground
    return walk_cfg(n, fix_base=fix_base, spawn_height=1.3 if fix_base else None)


def build(workload, n, seed, kinds):
    """(reference oracle, {kind: env}, action function of the reference obs, is_gogoro)."""
    gogoro = workload.startswith("gogoro")
    fix = workload.endswith("fixbase")
    runs = {}
    if gogoro:
        mk = lambda prec: OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), precision=prec, fix_base=fix)
        act = balance_policy
        if workload == "gogoro_random":
            rsa = np.random.default_rng(seed + 100)
            act = lambda o: rsa.uniform(-1, 1, (n, 1)).astype(np.float32)
    else:
        mk = lambda prec: OracleWalk(_walk_cfg(n, fix), NumpyDraws(seed), precision=prec)
        rs = np.random.default_rng(seed + 100)
        if workload == "walk_stand":
            act = lambda o: np.zeros((n, 33), np.float32)
        else:
            act = lambda o: rs.uniform(-0.3, 0.3, (n, 33)).astype(np.float32)
    ref = mk("f64")
    if "perturbed" in kinds:
        p = mk("f64")
        rs2 = np.random.default_rng(seed + 999)
        p.a["root"][:, 0:3] += (1e-6 * rs2.choice([-1.0, 1.0], (n, 3))).astype(np.float32)
        dof = p.a["dof_state"]
        dof[:, 0] += (1e-6 * rs2.choice([-1.0, 1.0], dof.shape[0])).astype(np.float32)
        runs["perturbed"] = p
    if "f32" in kinds:
        runs["f32"] = mk("f32")
    if "gpu" in kinds:
        if gogoro:
            from thormang_isaacgym_amd.tasks import gogoro as gmod
            saved, gmod.DEBUGFIXBASE = gmod.DEBUGFIXBASE, fix
            try:
                runs["gpu"] = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
            finally:
                gmod.DEBUGFIXBASE = saved
        else:
            runs["gpu"] = make_gpu_walk(_walk_cfg(n, fix), NumpyDraws(seed))
    return ref, runs, act, gogoro


def run(workload, steps, n, seed, kinds):
    import torch
    ref, runs, act_fn, gogoro = build(workload, n, seed, kinds)
    curves = {k: {"max": [], "median": [], "desync_envs": []} for k in runs}
    desync = {k: np.zeros(n, bool) for k in runs}
    obs = ref.a["obs_buf"].copy()
    t0 = time.time()
    for t in range(steps):
        act = act_fn(obs)
        o_act = act[:, 0] if gogoro else act
        r_obs, _, r_reset, _ = ref.step(o_act)
        r_obs, r_reset = r_obs.copy(), r_reset.copy()
        for k, env in runs.items():
            if k == "gpu":
                od, _, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
                g_obs, g_reset = od["obs"].cpu().numpy(), reset.cpu().numpy()
            else:
                g_obs, _, g_reset, _ = env.step(o_act)
            e = np.abs(g_obs - r_obs).max(axis=1)
            desync[k] |= g_reset != r_reset
            curves[k]["max"].append(float(e.max()))
            curves[k]["median"].append(float(np.median(e)))
            curves[k]["desync_envs"].append(int(desync[k].sum()))
        obs = r_obs
        if (t + 1) % 100 == 0:
            print(f"[{workload}] step {t + 1} ({time.time() - t0:.0f} s): " + ", ".join(
                f"{k} max {curves[k]['max'][-1]:.1e}" for k in runs), flush=True)
    out = {"workload": workload, "envs": n, "steps": steps, "seed": seed, "tol": TOL, "runs": {}}
    for k, c in curves.items():
        m = np.array(c["max"])
        bad = np.nonzero(m > TOL)[0]
        ds = np.nonzero(np.array(c["desync_envs"]) > 0)[0]
        out["runs"][k] = {"horizon": int(bad[0]) if bad.size else None,
                          "first_reset_desync": int(ds[0]) if ds.size else None,
                          "max_err_all_steps": float(m.max()), **c}
    return out


def table(out):
    lines = [f"# {out['workload']}: {out['envs']} envs, {out['steps']} steps, seed {out['seed']}; "
             f"max over envs of |obs - obs_fp64 oracle| per 50-step window (tol {out['tol']:g})"]
    ks = list(out["runs"])
    lines.append("steps        " + "".join(f"{k:>14s}" for k in ks))
    for w in range(0, out["steps"], 50):
        row = "".join(f"{max(out['runs'][k]['max'][w:w + 50]):14.2e}" for k in ks)
        lines.append(f"{w:4d}-{w + 49:4d}    {row}")
    lines.append("horizon (first step > tol): " + ", ".join(f"{k} {out['runs'][k]['horizon']}" for k in ks))
    lines.append("first reset-flag mismatch:  " + ", ".join(f"{k} {out['runs'][k]['first_reset_desync']}" for k in ks))
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["gogoro", "gogoro_random", "gogoro_fixbase", "walk", "walk_stand",
                                        "walk_fixbase"])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--seed", type=int, default=21)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--out", default="gpurun_out/drift")
    ap.add_argument("--kinds", default=None, help="comma list of perturbed,f32,gpu (default: all)")
    ap.add_argument("--label", default=None, help="name the gpu column gpu_<label>")
    ap.add_argument("--variants", default="", help="label=path.so,... extra GPU columns, one process each")
    a = ap.parse_args()
    kinds = a.kinds.split(",") if a.kinds else ["perturbed", "f32"] + ([] if a.no_gpu else ["gpu"])
    out = run(a.workload, a.steps, a.envs, a.seed, kinds)
    if a.label and "gpu" in out["runs"]:
        out["runs"]["gpu_" + a.label] = out["runs"].pop("gpu")
    for v in filter(None, a.variants.split(",")):
        import subprocess
        import tempfile
        label, lib = v.split("=", 1)
        with tempfile.TemporaryDirectory() as td:
            env = dict(os.environ, TG_LIB_PATH=os.path.abspath(lib))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), a.workload, "--steps", str(a.steps),
                                "--envs", str(a.envs), "--seed", str(a.seed), "--kinds", "gpu", "--label", label,
                                "--out", td], env=env)
            if r.returncode != 0:
                raise SystemExit(f"variant {label} failed ({r.returncode})")
            with open(os.path.join(td, f"drift_{a.workload}.json")) as f:
                out["runs"].update(json.load(f)["runs"])
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, f"drift_{a.workload}.json"), "w") as f:
        json.dump(out, f)
    t = table(out)
    with open(os.path.join(a.out, f"drift_{a.workload}.txt"), "w") as f:
        f.write(t + "\n")
    print(t)


if __name__ == "__main__":
    main()

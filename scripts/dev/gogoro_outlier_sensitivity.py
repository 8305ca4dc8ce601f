"""Developer probe: is the Gogoro 4096-env teacher-forced outlier (one
env-step whose base yaw rate, obs[2], the GPU gets 2.6e-4 away from the fp64
oracle while the fp32 oracle build is within 1e-7; scripts/dev/
gogoro_forced_outliers.py) a rounding-sensitive step?

save (GPU): run the teacher-forced scan to STEP and record the oracle's
inputs of that step (every buffer, the action, the draw generator's state),
the GPU's and the fp64 oracle's observations after it:

    python scripts/dev/gogoro_outlier_sensitivity.py save STEP ENV out.npz

study (CPU): replay that one step in the fp64 and the fp32 oracle from the
recorded inputs, unperturbed and with env ENV's root and joint state
perturbed by about one fp32 ulp (relative 1e-7, K draws), and print where the
GPU's yaw rate lies in the spread:

    python scripts/dev/gogoro_outlier_sensitivity.py study out.npz [K]
"""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.gpu_harness import NumpyDraws, OracleGogoro, parity_cfg, sync_oracle_from_gpu  # noqa: E402

n, seed = 4096, 23


def save(step, e, out):
    import torch
    from tests.gpu_harness import make_gpu_gogoro
    env = make_gpu_gogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed))
    orc = OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=16)
    rs = np.random.default_rng(n)
    for t in range(step + 1):
        sync_oracle_from_gpu(orc, env)
        act = rs.uniform(-1, 1, (n, 1)).astype(np.float32)
        if t == step:
            snap = {"a_" + k: v.copy() for k, v in orc.a.items()}
            state = json.dumps(orc.src.rs.bit_generator.state)
        od = env.step(torch.from_numpy(act).to("cuda:0"))[0]
        o_obs = orc.step(act[:, 0])[0].copy()
    np.savez(out, act=act, gpu_obs=od["obs"].cpu().numpy(), oracle_obs=o_obs, rng_state=np.array(state),
             step=step, env=e, **snap)
    print(f"step {step} env {e}: gpu obs {od['obs'][e].cpu().numpy()} oracle {o_obs[e]}")


def study(path, K):
    z = np.load(path)
    e, act = int(z["env"]), z["act"]
    state = json.loads(str(z["rng_state"]))
    snap = {k[2:]: z[k] for k in z.files if k.startswith("a_")}
    orcs = {p: OracleGogoro(parity_cfg(n, max_steps=1000), NumpyDraws(seed), threads=8, precision=p)
            for p in ("f64", "f32")}
    D = orcs["f64"].D
    rng = np.random.default_rng(99)

    def run(p, eps, pert=None, dump_sub=-1):
        orc = orcs[p]
        for k, v in snap.items():
            orc.a[k][...] = v
        orc.src.rs.bit_generator.state = state
        if eps:
            if pert is None:
                pert = (rng.standard_normal(13), rng.standard_normal((D, 2)))
            r = orc.a["root"][e]
            r[:] = r * (1 + eps * pert[0]).astype(np.float32)
            ds = orc.a["dof_state"][e * D:(e + 1) * D]
            ds[:] = ds * (1 + eps * pert[1]).astype(np.float32)
        if dump_sub >= 0:
            orc.L.oracle_dump_set.argtypes = [C.c_int, C.c_int]
            orc.L.oracle_dump_set(e, dump_sub)
        o = orc.step(act[:, 0])[0][e].copy()
        if dump_sub >= 0:
            buf = np.zeros(4096)
            orc.L.oracle_dump_read.argtypes = [C.c_void_p, C.c_int]
            orc.L.oracle_dump_read(buf.ctypes.data, 4096)
            orc.L.oracle_dump_set(-1, 0)
            return o, buf
        return o

    g = z["gpu_obs"][e]
    base = run("f64", 0.0)
    print(f"step {int(z['step'])} env {e}: yaw rate obs[2]  gpu {g[2]:.7f}  fp64 {base[2]:.7f} "
          f"(recorded {z['oracle_obs'][e][2]:.7f})  fp32 {run('f32', 0.0)[2]:.7f}")
    # which discrete decision flips: a perturbation that lands on the GPU's
    # value against the unperturbed replay, substep by substep (the oracle's
    # dump: drive-clamp flag and the nearest drive's distance to its effort
    # limit, multipliers)
    for _ in range(4 * K):
        pert = (rng.standard_normal(13), rng.standard_normal((D, 2)))
        if abs(run("f64", 1e-7, pert)[2] - base[2]) > 0.5 * abs(g[2] - base[2]):
            break
    for sub in range(3):
        for tag, pp in (("unperturbed", None), ("jumped     ", pert)):
            _, b = run("f64", 1e-7 if pp is not None else 0.0, pp, dump_sub=sub)
            k = int(b[0])
            print(f"  substep {sub} {tag}: drive clamp {int(b[2790])}, nearest drive dof {int(b[2792])} "
                  f"{b[2791]:.3e} from its effort limit; lam_pos {np.round(b[2600:2600 + k], 6)} "
                  f"lam_vel {np.round(b[2500:2500 + k], 6)}")
    for p in ("f64", "f32"):
        ys = np.array([run(p, 1e-7)[2] for _ in range(K)])
        d = ys - base[2]
        print(f"{p}, state x (1 + 1e-7 N(0,1)), {K} draws: yaw rate - unperturbed fp64: "
              f"min {d.min():+.3e} max {d.max():+.3e} std {d.std():.2e}; "
              f"|d| >= the GPU's {abs(g[2] - base[2]):.2e} in {int((np.abs(d) >= abs(g[2] - base[2])).sum())}/{K}")


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
    else:
        study(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 32)

"""Developer study: a GPU-only teacher-forced outlier of the DR walk
(scripts/dev/r6_walk_dr_probe.py: torch seed 1, step 58, env 13922 -- the
GPU's root 0.2 from fp64, the fp32 oracle build's 2.6e-5).  Is it a
discontinuity of the restated physics hit by rounding, or a kernel error?

  capture (GPU):  python scripts/dev/r6_walk_outlier.py capture STEP ENV TSEED
      replays the teacher-forced run to STEP and saves env ENV's physics
      inputs (after the pre-physics) and the GPU's result to
      gpurun_out/walk_outlier.npz
  replay (CPU):   python scripts/dev/r6_walk_outlier.py replay
      steps that one env in the fp64 and fp32 oracles, unperturbed and from
      48 states perturbed by ~1 fp32 ulp each, and reports where each lands
      against the GPU's result (a bimodal landing = a discontinuity)
"""
import sys

import numpy as np

sys.path.insert(0, ".")
OUT = "gpurun_out/walk_outlier.npz"


def capture(step, e, tseed, n=16384, seed=12):
    import torch
    from tests.gpu_harness import NumpyDraws, OracleWalk, make_gpu_walk, sync_dr, sync_oracle_from_gpu, walk_cfg
    mk = lambda: walk_cfg(n, "ThormangWalkDR", dr=True)
    env = make_gpu_walk(mk(), NumpyDraws(seed), torch_seed=tseed)
    orc = OracleWalk(mk(), NumpyDraws(seed))
    rs = np.random.default_rng(seed + 100)
    D = orc.D
    for t in range(step + 1):
        sync_oracle_from_gpu(orc, env)
        sync_dr(orc, env)
        act = rs.uniform(-0.5, 0.5, (n, D)).astype(np.float32)
        if t == step:
            import ctypes as C
            from tests.oracle_lib import ptr
            a = orc.a
            orc.L.oracle_walk_pre_physics(C.byref(orc.p), C.byref(orc.b), ptr(np.ascontiguousarray(act)))
            cap = dict(root=a["root"][e].copy(), dof=a["dof_state"][e * D:(e + 1) * D].copy(),
                       props=orc.props[:, e, :].copy(), pos_target=a["pos_target"][e].copy(),
                       force=(a["body_force"][e].copy() if orc.push else np.zeros(0, np.float32)),
                       mass_scale=orc.dr["mass_scale"][e].copy(), mu=orc.dr["mu"][e].copy(),
                       gravity=np.asarray(orc.dr["gravity"], np.float32))
        env.step(torch.from_numpy(act).to("cuda:0"))
        if t < step:
            orc.step(act)
    cap["gpu_root"] = env.root_tensor[e].cpu().numpy()
    cap["gpu_dof"] = env.sim.dof_state.view(n, D, 2)[e].cpu().numpy()
    np.savez(OUT, **cap)
    print("captured", {k: v.shape for k, v in cap.items()})


def replay():
    from tests.gpu_harness import walk_cfg
    from tests.oracle_lib import lib, physics_step
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.tasks.thormang_walk import load_model, walk_asset_options, walk_model_name
    c = dict(np.load(OUT))
    cfg = walk_cfg(1, "ThormangWalkDR", dr=True)
    m = load_model(walk_model_name(cfg))
    desc = abi.ModelDesc(m)
    sp = abi.sim_params_from_cfg(cfg["sim"], walk_asset_options(cfg), 1, float(cfg["env"].get("envSpacing", 1.0)),
                                 default_contact_offset=0.016)
    D = m.num_dof

    def one(prec, root, dof):
        r, d = root[None].copy(), dof.copy()
        force = c["force"][None] if c["force"].size else None
        physics_step(desc, sp, r, d, np.ascontiguousarray(c["props"][:, None, :]), c["pos_target"][None].copy(),
                     np.zeros((1, D), np.float32), force=force, mass_scale=c["mass_scale"][None].copy(),
                     mu=c["mu"][None].copy(), gravity=c["gravity"], L=lib(prec))
        return r[0]

    g = c["gpu_root"]
    np.set_printoptions(precision=6, suppress=True, linewidth=200)
    print("gpu   ", g)
    for prec in ("f64", "f32"):
        r0 = one(prec, c["root"], c["dof"])
        print(f"{prec} unperturbed", r0, "| max |gpu - it|", float(np.abs(g - r0).max()))
    rs = np.random.default_rng(5)
    for prec in ("f64", "f32"):
        near, far, dists = 0, 0, []
        for k in range(48):
            root = c["root"] * (1 + rs.choice([-1, 1], 13) * 1.2e-7).astype(np.float32)
            dof = c["dof"] * (1 + rs.choice([-1, 1], c["dof"].shape) * 1.2e-7).astype(np.float32)
            r = one(prec, root.astype(np.float32), dof.astype(np.float32))
            dg = float(np.abs(r - g).max())
            dists.append(dg)
            near += dg < 1e-2
        print(f"{prec}: 48 perturbed replays, within 1e-2 of the GPU's root: {near}; "
              f"distances min {min(dists):.2e} median {np.median(dists):.2e} max {max(dists):.2e}")


if __name__ == "__main__":
    if sys.argv[1] == "capture":
        capture(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
    else:
        replay()

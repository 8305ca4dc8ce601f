"""Developer probe (GPU): the yaw rate of boxes spinning on the ground (the
torsional friction row of a 4-point patch), GPU and the fp32 oracle build
each against the fp64 oracle, teacher-forced one step at a time from the
fp64 state; prints the max error of every root-state component."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests import physics_models as pm  # noqa: E402
from tests.oracle_lib import lib, physics_step  # noqa: E402
from tests.test_gpu_physics import gpu_sim  # noqa: E402

for solver in (0, 1):
    n = 256
    st = pm.sim(pm.box_body(), n=n, dt=1 / 60, substeps=2, solver_type=solver, contact_iterations=4, velocity_iterations=1)
    desc, sp, root, dof, props, pt, vt = st
    rs = np.random.default_rng(0)
    root[:, 2] = 0.05 + rs.uniform(-0.002, 0.004, n)
    yaw = rs.uniform(-np.pi, np.pi, n)
    root[:, 5], root[:, 6] = np.sin(yaw / 2), np.cos(yaw / 2)
    root[:, 7:9] = rs.normal(0, 0.3, (n, 2))
    root[:, 12] = rs.uniform(-4, 4, n)
    g = gpu_sim(pm.box_body(), sp, n, root, dof, props, pt, vt)
    eg = np.zeros(13)
    ec = np.zeros(13)
    for t in range(60):
        g.root_state.copy_(__import__("torch").from_numpy(root).cuda())
        r32 = root.copy()
        physics_step(desc, sp, r32, dof.copy(), props, pt, vt, L=lib("f32"))
        physics_step(desc, sp, root, dof, props, pt, vt)
        g.simulate()
        gr = g.root_state.cpu().numpy()
        eg = np.maximum(eg, np.abs(gr - root).max(0))
        ec = np.maximum(ec, np.abs(r32 - root).max(0))
    np.set_printoptions(precision=1)
    print(f"solver {solver}: gpu  err per root component", eg)
    print(f"solver {solver}: fp32 err per root component", ec)

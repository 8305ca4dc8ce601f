"""CPU tests of the standing-walk yardstick (tests/gpu_harness.py
perturbed_walk_oracle, used by the fp32 ensembles of tests/test_gpu_parity_seeds.py):
the perturbation is a rounding-level, reproducible change of the initial
state, and it leaves the reference's first steps inside the 1e-3 band."""
import numpy as np

from tests.gpu_harness import NumpyDraws, OracleWalk, perturbed_walk_oracle, walk_cfg


def test_perturbation_is_rounding_level_and_reproducible():
    ref = OracleWalk(walk_cfg(4), NumpyDraws(21))
    a = perturbed_walk_oracle(walk_cfg(4), 21, 0)
    b = perturbed_walk_oracle(walk_cfg(4), 21, 0)
    c = perturbed_walk_oracle(walk_cfg(4), 21, 1)
    dz = np.abs(a.a["root"][:, 2] - ref.a["root"][:, 2])
    dq = np.abs(a.a["dof_state"][:, 0] - ref.a["dof_state"][:, 0])
    assert 0 < dz.max() < 1e-6 and 0 < dq.max() < 1e-6          # fp32 storage rounds 1e-7 to an ulp
    assert np.array_equal(a.a["root"], b.a["root"]) and np.array_equal(a.a["dof_state"], b.a["dof_state"])
    assert not np.array_equal(a.a["dof_state"], c.a["dof_state"])   # stream k is its own sign pattern
    np.testing.assert_array_equal(a.a["root"][:, :2], ref.a["root"][:, :2])   # x, y untouched


def test_perturbed_reference_stays_in_band_at_first():
    n = 4
    ref = OracleWalk(walk_cfg(n), NumpyDraws(21))
    p = perturbed_walk_oracle(walk_cfg(n), 21, 0)
    act = np.zeros((n, ref.D), np.float32)
    worst = 0.0
    for _ in range(20):
        r_obs = ref.step(act)[0].copy()
        p_obs = p.step(act)[0]
        worst = max(worst, float(np.abs(p_obs - r_obs).max()))
    assert 0.0 < worst < 1e-4, worst

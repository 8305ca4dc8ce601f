"""Terrain on the CPU: the restated Perlin field against the
reference's own output (tests/golden/terrain.npz, make_golden_terrain.py), the
trimesh triangulation against the surface the contact code evaluates, and the
oracle's heightfield contact against closed-form incline answers.

The mesh triangulation is isaacgym's convert_heightfield_to_trimesh, which the
reference imports but does not contain: its layout here is restated from the
published isaacgym terrain_utils (parity unpinned by a fixture; checked for
self-consistency below)."""
import os

import numpy as np
import pytest
import torch

from thormang_isaacgym_amd.tasks import terrain as tt

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "terrain.npz")


def test_perlin_matches_reference_bitwise():
    f = np.load(GOLDEN)
    for k in range(3):
        nx, ny, rx, ry, octv, pers, seed = f[f"small{k}_cfg"]
        torch.manual_seed(int(seed))
        got = tt.perlin_2d_octaves((int(nx), int(ny)), (int(rx), int(ry)), int(octv), float(pers)).numpy()
        np.testing.assert_array_equal(got, f[f"small{k}"])


@pytest.mark.parametrize("seed", [0, 42])
def test_terrain_matches_reference(seed):
    f = np.load(GOLDEN)
    torch.manual_seed(seed)
    hs = tt.Terrain().heightsamples.numpy()
    assert hs.shape == (512, 512)
    np.testing.assert_array_equal(hs[::4, ::4], f[f"full{seed}_sub4"])
    np.testing.assert_array_equal(hs.astype(np.float64).sum(1), f[f"full{seed}_rowsum"])
    assert hs.astype(np.float64).sum() == float(f[f"full{seed}_sum"])


def test_explicit_generator_equals_global_stream():
    torch.manual_seed(5)
    a = tt.perlin_2d_octaves((64, 64), (1, 4), 2).numpy()
    g = torch.Generator().manual_seed(5)
    b = tt.perlin_2d_octaves((64, 64), (1, 4), 2, generator=g).numpy()
    np.testing.assert_array_equal(a, b)


def test_trimesh_surface_is_the_evaluated_surface():
    """Every triangle of the mesh, sampled at random barycentric points, lies
    on Terrain.height_at (the formula the kernel and the oracle use)."""
    rs = np.random.default_rng(0)
    t = tt.Terrain(torch.Generator().manual_seed(3), shape=(16, 32), with_mesh=True)
    v, tri = t.vertices.astype(np.float64), t.triangles
    assert v.shape == (16 * 32, 3) and tri.shape == (2 * 15 * 31, 3)
    w = rs.dirichlet([1, 1, 1], size=tri.shape[0])
    p = np.einsum("tk,tkj->tj", w, v[tri])
    np.testing.assert_allclose(t.height_at(p[:, 0], p[:, 1]), p[:, 2], atol=2e-6)
    # every triangle is counter-clockwise seen from above (upward normals)
    a, b, c = v[tri[:, 0]], v[tri[:, 1]], v[tri[:, 2]]
    assert (np.cross(b - a, c - a)[:, 2] > 0).all()


# ------------------------------------------------------------------ oracle terrain contact
def _incline(theta, n=8):
    """A heightfield plane z = tan(theta) * x over [0, 40] x [0, 40] m."""
    hs = 0.5
    x = np.arange(n * 10) * hs
    return np.repeat((np.tan(theta) * x)[:, None], n * 10, 1).astype(np.float32), hs


def _box_on_incline(theta, mu, steps):
    from tests import physics_models as pm
    from tests.oracle_lib import physics_step, set_heightfield
    h, hs = _incline(theta)
    desc, sp, root, dof, props, pt, vt = pm.sim(pm.box_body(mu=mu), dt=0.005, substeps=1, ground_friction=mu)
    x0, half = 20.0, 0.05
    # rest the box on the slope: rotated about y by -theta, centre half a box above the surface along n
    n = np.array([-np.sin(theta), 0.0, np.cos(theta)])
    root[0, :3] = np.array([x0, 20.0, np.tan(theta) * x0]) + half * n
    root[0, 3:7] = [0.0, np.sin(-theta / 2), 0.0, np.cos(-theta / 2)]
    root[0, 7:] = 0
    set_heightfield(h, hs, 1.0, 0.0, 0.0, friction=mu)
    try:
        traj = []
        for _ in range(steps):
            physics_step(desc, sp, root, dof, props, pt, vt)
            traj.append(root[0].copy())
    finally:
        set_heightfield(None)
    return np.array(traj), sp


@pytest.mark.parametrize("theta", [0.15, 0.3])
def test_oracle_box_sticks_on_incline_when_mu_exceeds_slope(theta):
    traj, sp = _box_on_incline(theta, mu=np.tan(theta) + 0.4, steps=120)
    drift = np.linalg.norm(traj[-1, :3] - traj[0, :3])
    assert drift < 2e-3, drift
    assert np.abs(traj[-1, 7:13]).max() < 2e-2


@pytest.mark.parametrize("theta", [0.2, 0.35])
def test_oracle_box_slides_down_incline_at_g_sin_minus_mu_cos(theta):
    mu = 0.1
    traj, sp = _box_on_incline(theta, mu=mu, steps=90)
    dt = sp.dt
    g = abs(sp.gravity[2])
    # speed along the slope (down = -x direction along the incline)
    d = np.array([-np.cos(theta), 0.0, -np.sin(theta)])
    v = traj[:, 7:10] @ d
    k0, k1 = 30, 89
    acc = (v[k1] - v[k0]) / ((k1 - k0) * dt)
    expect = g * (np.sin(theta) - mu * np.cos(theta))
    assert abs(acc - expect) < 0.03 * expect + 0.05, (acc, expect)
    # stays on the surface: height above the incline ~ constant
    c = traj[:, :3]
    nrm = np.array([-np.sin(theta), 0.0, np.cos(theta)])
    gap = (c - np.array([0.0, 0.0, 0.0])) @ nrm
    assert np.ptp(gap[k0:]) < 5e-3


def test_oracle_flat_heightfield_equals_plane():
    """A heightfield at constant height z0 behaves like the plane lifted by z0."""
    from tests import physics_models as pm
    from tests.oracle_lib import physics_step, set_heightfield
    z0 = 0.75
    outs = []
    for use_hf in (False, True):
        desc, sp, root, dof, props, pt, vt = pm.sim(pm.box_body(mu=0.6), dt=0.005, ground_friction=0.6)
        root[0, :3] = [3.3, 2.1, 0.3 + (z0 if use_hf else 0.0)]
        root[0, 3:7] = [0.1, 0.05, 0.0, np.sqrt(1 - 0.0125)]
        root[0, 7:10] = [0.4, -0.2, 0.0]
        if use_hf:
            set_heightfield(np.full((20, 20), z0, np.float32), 0.5, 1.0, 0.0, 0.0, friction=0.6)
        try:
            for _ in range(150):
                physics_step(desc, sp, root, dof, props, pt, vt)
        finally:
            set_heightfield(None)
        r = root[0].copy()
        if use_hf:
            r[2] -= z0
        outs.append(r)
    assert outs[0][2] < 0.1            # it landed
    np.testing.assert_allclose(outs[1], outs[0], atol=1e-5)

"""Perlin terrain of the Gogoro task.

The reference builds, when ``USE_TERAIN`` is set (tasks/gogoro_new.py:26,157),
a 512 x 512 Perlin heightfield (``Terrain``, gogoro_new.py:734-790), turns it
into a triangle mesh with ``isaacgym.terrain_utils.convert_heightfield_to_trimesh``
and adds that mesh beside the z = 0 plane (gogoro_new.py:164-181).  Here:

* ``perlin_2d`` / ``perlin_2d_octaves`` -- the reference's gradient noise
  (gogoro_new.py:761-790), drawing its lattice angles with ``torch.rand`` on
  the CPU generator in the same order, so a given ``torch.manual_seed`` gives
  the reference's terrain bit for bit (tests/golden/terrain.npz);
* ``Terrain`` -- the 512 x 512 field, its edge ramp and scales (:734-758);
* ``heightfield_to_trimesh`` -- the published isaacgym terrain_utils
  triangulation (not vendored in the reference; restated),
  kept for API users that want the mesh.  The simulator itself is handed the
  height samples (``Sim.set_heightfield``) and evaluates exactly that mesh's
  surface in the contact kernel, so no triangle soup is uploaded.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _fade(t):
    # quintic smoothstep 6t^5 - 15t^4 + 10t^3 (same fp32 evaluation order as the reference)
    return 6 * t ** 5 - 15 * t ** 4 + 10 * t ** 3


def perlin_2d(shape, res, generator: torch.Generator | None = None) -> torch.Tensor:
    """Gradient noise on a ``res`` lattice sampled on a ``shape`` grid
    (gogoro_new.py:761-777).  ``shape`` must be a multiple of ``res``."""
    nx, ny = shape
    rx, ry = res
    cx, cy = nx // rx, ny // ry                    # samples per lattice cell
    # fractional position of every sample inside its cell
    fx = torch.arange(0, rx, rx / nx)[:nx] % 1
    fy = torch.arange(0, ry, ry / ny)[:ny] % 1
    gxf, gyf = torch.meshgrid(fx, fy, indexing="ij")
    ang = 2 * math.pi * torch.rand(rx + 1, ry + 1, generator=generator)
    gcos, gsin = torch.cos(ang), torch.sin(ang)
    ci = torch.arange(nx) // cx                    # lattice cell of each sample
    cj = torch.arange(ny) // cy

    def corner(di, dj, sx, sy):
        ii, jj = (ci + di)[:, None], (cj + dj)[None, :]
        return (gxf + sx) * gcos[ii, jj] + (gyf + sy) * gsin[ii, jj]

    n00 = corner(0, 0, 0, 0)
    n10 = corner(1, 0, -1, 0)
    n01 = corner(0, 1, 0, -1)
    n11 = corner(1, 1, -1, -1)
    tx, ty = _fade(gxf), _fade(gyf)
    return math.sqrt(2) * torch.lerp(torch.lerp(n00, n10, tx), torch.lerp(n01, n11, tx), ty)


def perlin_2d_octaves(shape, res, octaves: int = 1, persistence: float = 0.5,
                      generator: torch.Generator | None = None) -> torch.Tensor:
    """Sum of ``octaves`` noise layers, lattice 2x finer and amplitude x
    persistence per layer, starting at 2 x res (gogoro_new.py:780-790)."""
    noise = torch.zeros(shape)
    freq, amp = 2, 1
    for _ in range(octaves):
        noise += amp * perlin_2d(shape, (freq * res[0], freq * res[1]), generator)
        freq *= 2
        amp *= persistence
    return noise


def edge_ramp(nx: int, ny: int, width: float = 10.0) -> torch.Tensor:
    """min(distance to the border in samples / width, 1) (gogoro_new.py:747-755)."""
    i = torch.arange(nx).view(nx, 1).expand(nx, ny)
    j = torch.arange(ny).view(1, ny).expand(nx, ny)
    d = torch.min(torch.min(i, nx - 1 - i), torch.min(j, ny - 1 - j)) / width
    return d.clamp(max=1.0)


def heightfield_to_trimesh(heights: np.ndarray, horizontal_scale: float, vertical_scale: float):
    """isaacgym.terrain_utils.convert_heightfield_to_trimesh (slope_threshold
    None): vertex (i, j) -> (i hs, j hs, h[i, j] vs); cell (i, j) ->
    triangles (i,j)-(i+1,j+1)-(i,j+1) and (i,j)-(i+1,j)-(i+1,j+1)."""
    h = np.asarray(heights)
    r, c = h.shape
    ii, jj = np.meshgrid(np.arange(r), np.arange(c), indexing="ij")
    vertices = np.stack([ii.ravel() * horizontal_scale, jj.ravel() * horizontal_scale,
                         h.ravel() * vertical_scale], 1).astype(np.float32)
    v00 = (np.arange(r - 1)[:, None] * c + np.arange(c - 1)[None, :]).ravel()
    tri = np.empty((2 * v00.size, 3), np.uint32)
    tri[0::2] = np.stack([v00, v00 + c + 1, v00 + 1], 1)
    tri[1::2] = np.stack([v00, v00 + c, v00 + c + 1], 1)
    return vertices, tri


class Terrain:
    """The Gogoro task's terrain (gogoro_new.py:734-758): 512 x 512 samples,
    0.5 m apart, unit height scale, 2 octaves of Perlin noise on a (1, 4)
    base lattice, lifted by 0.1 and ramped to zero over the outer 10 samples.
    Random angles come from the CPU torch generator (global by default)."""

    def __init__(self, generator: torch.Generator | None = None, shape=(512, 512), v_scale: float = 0.5,
                 h_scale: float = 1.0, with_mesh: bool = False):
        self.Vx_shape, self.Vy_shape = shape
        self.V_scale = v_scale
        self.H_scale = h_scale
        self.Vx_size_m = self.V_scale * self.Vx_shape
        self.Vy_size_m = self.V_scale * self.Vy_shape
        ramp = edge_ramp(self.Vx_shape, self.Vy_shape)
        noise = perlin_2d_octaves(shape, (1, 4), 2, generator=generator)
        self.heightsamples = (noise + 0.1) * ramp
        self.vertices = self.triangles = None
        if with_mesh:
            self.vertices, self.triangles = heightfield_to_trimesh(self.heightsamples.numpy(), self.V_scale,
                                                                   self.H_scale)

    def height_at(self, x, y):
        """Mesh height at terrain-frame (x, y) (before the max with the z = 0 plane)."""
        return surface_height(self.heightsamples, self.V_scale, self.H_scale, x, y)


def surface_height(heights, horizontal_scale: float, vertical_scale: float, x, y):
    """Height of the heightfield trimesh at terrain-frame (x, y), in float64 --
    the surface tg_set_heightfield's contact code evaluates (inside the grid;
    before the max with the z = 0 plane)."""
    if isinstance(heights, torch.Tensor):
        heights = heights.detach().cpu().numpy()
    h = np.asarray(heights, np.float64) * vertical_scale
    u, v = np.asarray(x, np.float64) / horizontal_scale, np.asarray(y, np.float64) / horizontal_scale
    i = np.clip(u.astype(np.int64), 0, h.shape[0] - 2)
    j = np.clip(v.astype(np.int64), 0, h.shape[1] - 2)
    fu, fv = u - i, v - j
    h00, h01, h10, h11 = h[i, j], h[i, j + 1], h[i + 1, j], h[i + 1, j + 1]
    return np.where(fu >= fv, h00 + fu * (h10 - h00) + fv * (h11 - h10),
                    h00 + fu * (h11 - h01) + fv * (h01 - h00))

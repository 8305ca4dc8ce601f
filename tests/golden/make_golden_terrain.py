"""Generate tests/golden/terrain.npz: the reference's Perlin terrain.

RUNS ONLY IN THE BUILD CONTAINER (needs /root/reference).  Imports the
reference's ``tasks/gogoro_new.py`` through make_golden.load_reference() and
records, for fixed ``torch.manual_seed`` values:

* ``Terrain.rand_perlin_2d_octaves`` (gogoro_new.py:780-790) on small grids
  (full arrays) -- pins the noise function including its RNG call order;
* a full ``Terrain()`` (gogoro_new.py:734-758, 512 x 512 with the edge ramp):
  every 4th sample, the float64 sum and the per-row sums of all samples.

``isaacgym.terrain_utils.convert_heightfield_to_trimesh`` is not part of the
reference (its terrain_utils is an isaacgym module); the constructor's call is
stubbed to return nothing, so only the height samples are recorded.  Data only
leaves the container.  Re-run:  python tests/golden/make_golden_terrain.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main():
    from make_golden import load_reference
    _, gg = load_reference()
    gg.convert_heightfield_to_trimesh = lambda *a, **k: (None, None)
    T = gg.Terrain
    obj = T.__new__(T)
    out = {}
    small = [((64, 64), (1, 4), 2, 0.5, 11), ((32, 128), (2, 1), 1, 0.5, 12), ((48, 96), (1, 2), 3, 0.7, 13)]
    for k, (shape, res, octv, pers, seed) in enumerate(small):
        torch.manual_seed(seed)
        out[f"small{k}_cfg"] = np.array([*shape, *res, octv, pers, seed], np.float64)
        out[f"small{k}"] = obj.rand_perlin_2d_octaves(shape, res, octv, pers).numpy()
    for seed in (0, 42):
        torch.manual_seed(seed)
        hs = T().heightsamples.numpy()
        out[f"full{seed}_sub4"] = hs[::4, ::4].copy()
        out[f"full{seed}_sum"] = np.array(hs.astype(np.float64).sum())
        out[f"full{seed}_rowsum"] = hs.astype(np.float64).sum(1)
    np.savez_compressed(os.path.join(HERE, "terrain.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

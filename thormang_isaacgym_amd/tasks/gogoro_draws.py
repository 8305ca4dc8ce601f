"""Replay-mode random draws for the Gogoro task.

The fused kernels draw their own noise (Philox, in-kernel) on the fast path.
For parity with the reference -- whose draws are ``torch.rand``/``torch.randn``
calls in a fixed order -- a ``DrawSource`` can be
attached; these helpers pull raw draws from it in exactly the reference's call
order and scatter them into the per-env arrays the kernels accept
(include/tg_gogoro.h):

* pre_physics_step: ``randn(N)``                      (tasks/gogoro_new.py:362)
* reset_idx(ids), k = len(ids):                        (:474-591)
    rand(k) speed, randn(k) steer offset, rand(k) speed offset    (randomize :479-482)
    rand(k) spawn target, rand(k) spawn yaw offset               (generate_spawn_r :486-487)
    randn(k) x5 config vector                                     (:554-559)
    rand(1) per env, in id order: steering damping               (:577)
* compute_obs_rwd: ``randn(N)`` x5                      (:451-460)
* resampling: ``rand(#speed changes)``, ``rand(N)``      (:386-387)

A DrawSource exposes ``uniform(n)`` and ``normal(n)`` returning raw float32
numpy arrays (U[0,1) and N(0,1) before the task's affine maps)."""
from __future__ import annotations

import numpy as np

RESET_DRAWS = 11


def reset_draws(src, ids: np.ndarray, n_envs: int) -> np.ndarray:
    """Raw reset draws [N,11] for the envs in ``ids`` (ascending), rows of other envs zero."""
    k = len(ids)
    out = np.zeros((n_envs, RESET_DRAWS), np.float32)
    if k == 0:
        return out
    out[ids, 0] = src.uniform(k)
    out[ids, 1] = src.normal(k)
    out[ids, 2] = src.uniform(k)
    out[ids, 3] = src.uniform(k)
    out[ids, 4] = src.uniform(k)
    for c in range(5):
        out[ids, 5 + c] = src.normal(k)
    for i in ids:
        out[i, 10] = src.uniform(1)[0]
    return out


def post_draws(src, reset_ids: np.ndarray, progress_prev: np.ndarray, speed_freq: int, yaw_freq: int):
    """All draws of one Gogoro.post_physics_step, returned as kernel arrays
    (reset_draws [N,11], obs_draws [N,5], speed_draws [N], yaw_draws [N])."""
    n = progress_prev.shape[0]
    rd = reset_draws(src, reset_ids, n)
    od = np.stack([src.normal(n) for _ in range(5)], 1).astype(np.float32)
    prog = progress_prev + 1
    prog[reset_ids] = 0
    speed_ids = np.nonzero(prog == speed_freq)[0]
    sd = np.zeros(n, np.float32)
    sd[speed_ids] = src.uniform(len(speed_ids))
    yd = src.uniform(n).astype(np.float32)
    return rd, od, sd, yd


class RecordedDraws:
    """DrawSource over a recorded stream (kinds 0=uniform, 1=normal; sizes; values).
    Verifies that every request matches the recorded kind and size -- i.e. that
    the caller reproduces the reference's RNG call order exactly."""

    def __init__(self, kinds, sizes, vals):
        self.kinds, self.sizes = np.asarray(kinds), np.asarray(sizes)
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)])
        self.vals = np.asarray(vals, np.float32)
        self.i = 0

    def _take(self, kind, n):
        if self.i >= len(self.kinds):
            raise AssertionError(f"draw stream exhausted at request {kind}({n})")
        k, s = int(self.kinds[self.i]), int(self.sizes[self.i])
        if k != kind or s != n:
            raise AssertionError(f"draw #{self.i}: expected {'normal' if k else 'uniform'}({s}), "
                                 f"got {'normal' if kind else 'uniform'}({n})")
        v = self.vals[self.offsets[self.i]:self.offsets[self.i + 1]]
        self.i += 1
        return v.copy()

    def uniform(self, n):
        return self._take(0, n)

    def normal(self, n):
        return self._take(1, n)

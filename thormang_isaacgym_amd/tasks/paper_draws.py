"""Replay-mode random draws for the Gogoro "paper" variant.

Pulls raw U[0,1) draws from a DrawSource in the reference's call order
(tasks/gogoro_realistic_turning_sim_paper.py) and scatters them into the
per-env arrays of include/tg_gogoro_paper.h:

* constructor (:75-90): rand(N) speed, steer offset, steer delay, steering
  damping, speed-sensor offset, imu x offset                 -> ctor_draws [N,6]
* reset_idx(ids), k = len(ids) (:609-692):
    rand(k) speed, delay, steer offset, speed offset          (randomize :565-575)
    per id, ascending: rand(1) imu x offset
                       [RANDOM_DAMPING] rand(1) steering damping
                       [not CENTER_ROBOT] rand(1) seat x, y, z   -> reset_draws [N,9]
* compute_obs_rwd (:521-527): rand(N,2) imu filter, rand(N,2) imu,
  rand(N) speed noise, rand(N) delta-yaw filter               -> noise_draws [N,6]
* command changes (:410-413): rand(#speed changes), rand(N)   -> speed [N], yaw [N]
* pushes (:446-447, PUSH_ROBOT): rand(N) x, rand(N) z           -> push_draws [N,2]
"""
from __future__ import annotations

import numpy as np

RESET_DRAWS = 9


def ctor_draws(src, n: int) -> np.ndarray:
    return np.stack([src.uniform(n) for _ in range(6)], 1).astype(np.float32)


def reset_draws(src, ids: np.ndarray, n_envs: int, random_damping: bool, center_robot: bool) -> np.ndarray:
    out = np.zeros((n_envs, RESET_DRAWS), np.float32)
    k = len(ids)
    if k == 0:
        return out
    for c in range(4):
        out[ids, c] = src.uniform(k)
    for i in ids:
        out[i, 4] = src.uniform(1)[0]
        if random_damping:
            out[i, 5] = src.uniform(1)[0]
        if not center_robot:
            for c in range(3):
                out[i, 6 + c] = src.uniform(1)[0]
    return out


def post_draws(src, reset_ids: np.ndarray, progress_prev: np.ndarray, speed_freq: int, push: bool,
               random_damping: bool, center_robot: bool):
    n = progress_prev.shape[0]
    rd = reset_draws(src, reset_ids, n, random_damping, center_robot)
    nd = np.zeros((n, 6), np.float32)
    nd[:, 0:2] = src.uniform(2 * n).reshape(n, 2)
    nd[:, 2:4] = src.uniform(2 * n).reshape(n, 2)
    nd[:, 4] = src.uniform(n)
    nd[:, 5] = src.uniform(n)
    prog = progress_prev + 1
    prog[reset_ids] = 0
    speed_ids = np.nonzero(prog == speed_freq)[0]
    sd = np.zeros(n, np.float32)
    sd[speed_ids] = src.uniform(len(speed_ids))
    yd = src.uniform(n).astype(np.float32)
    pd = np.zeros((n, 2), np.float32)
    if push:
        pd[:, 0] = src.uniform(n)
        pd[:, 1] = src.uniform(n)
    return rd, nd, sd, yd, pd

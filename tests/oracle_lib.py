"""ctypes loader for the CPU oracle (oracle/_build/liboracle.so) -- test infrastructure.

Builds the oracle with ``make -C oracle`` on first use if the shared object is
missing.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "_build", "liboracle.so")
LIB_F32 = os.path.join(REPO, "oracle", "_build", "liboracle_f32.so")   # physics in fp32 (drift study)

_libs = {}


def lib(precision: str = "f64"):
    """The oracle library: ``f64`` (the parity oracle) or ``f32`` (the same
    physics restatement evaluated in float, scripts/parity_drift.py)."""
    if precision not in _libs:
        path = {"f64": LIB, "f32": LIB_F32}[precision]
        srcs = [os.path.join(REPO, "oracle", f) for f in ("gogoro_task.c", "gogoro_paper_task.c", "physics_ref.c",
                                                              "walk_task.c")]
        if not os.path.exists(path) or any(os.path.getmtime(s) > os.path.getmtime(path) for s in srcs):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, capture_output=True)
        _lib = C.CDLL(path)
        vp = C.c_void_p
        _lib.oracle_gogoro_observations.argtypes = [C.c_int, vp, vp, vp, vp]
        _lib.oracle_gogoro_reward.argtypes = [C.c_int, vp, vp, vp, C.c_int64, vp, vp]
        _lib.oracle_gogoro_pre_physics.argtypes = [vp, vp, vp, vp]
        _lib.oracle_gogoro_post_physics.argtypes = [vp, vp, vp, vp, vp, vp]
        _lib.oracle_walk_pre_physics.argtypes = [vp, vp, vp]
        _lib.oracle_walk_post_physics.argtypes = [vp, vp, vp, vp]
        _lib.oracle_walk_reset_env.argtypes = [vp, vp, C.c_int, vp]
        _lib.oracle_paper_pre_physics.argtypes = [vp, vp, vp]
        _lib.oracle_paper_reset_env.argtypes = [vp, vp, C.c_int, vp]
        _lib.oracle_paper_post_physics.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        _lib.oracle_paper_head_wrench.argtypes = [vp, vp]
        _lib.oracle_paper_observation.argtypes = [vp, C.c_float, C.c_float, C.c_float, vp]
        _lib.oracle_physics_step.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int]
        _lib.oracle_set_heightfield.argtypes = [vp, C.c_int, C.c_int] + [C.c_float] * 5
        _lib.oracle_rigid_body_states.argtypes = [vp, C.c_int, vp, vp, vp]
        _lib.oracle_rigid_body_force_wrench.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp]
        _lib.oracle_gogoro_reset_env.argtypes = [vp, vp, C.c_int, vp]
        _libs[precision] = _lib
    return _libs[precision]


def ptr(a):
    if a is None:
        return None
    assert isinstance(a, np.ndarray) and a.flags.c_contiguous, "oracle arrays must be C-contiguous numpy"
    return a.ctypes.data_as(C.c_void_p)


def physics_step(desc, sp, root, dof, props, pos_tgt, vel_tgt, act=None, force=None, mass_scale=None, mu=None,
                 gravity=None, threads=1, L=None):
    """One control step of the fp64 oracle engine, in place on root/dof."""
    n = root.shape[0]
    if mu is None:
        mu = np.ascontiguousarray(np.broadcast_to(desc.arrays["shape_friction"], (n, len(desc.arrays["shape_friction"]))),
                                  dtype=np.float32)
    if gravity is None:
        gravity = np.array(list(sp.gravity), np.float32)
    (L or lib()).oracle_physics_step(C.byref(desc.desc), C.byref(sp), n, ptr(root), ptr(dof), ptr(props), ptr(pos_tgt),
                              ptr(vel_tgt), ptr(act), ptr(force), ptr(mass_scale), ptr(mu), ptr(gravity), threads)


_hf_keep = None   # the oracle keeps a pointer: hold the array while it is set


def set_heightfield(heights, horizontal_scale=1.0, vertical_scale=1.0, origin_x=0.0, origin_y=0.0, friction=1.0):
    """The oracle's terrain (tg_set_heightfield semantics); None = flat plane only."""
    global _hf_keep
    if heights is None:
        lib().oracle_set_heightfield(None, 0, 0, 1.0, 1.0, 0.0, 0.0, 1.0)
        _hf_keep = None
        return
    _hf_keep = np.ascontiguousarray(np.asarray(heights, np.float32))
    r, c = _hf_keep.shape
    lib().oracle_set_heightfield(ptr(_hf_keep), r, c, horizontal_scale, vertical_scale, origin_x, origin_y, friction)


def rigid_body_states(desc, root, dof):
    """[N, L, 13] world link states from root [N,13] / dof [N*D,2] (tg_rigid_body_states semantics)."""
    n = root.shape[0]
    out = np.zeros((n, desc.model.num_bodies, 13), np.float32)
    lib().oracle_rigid_body_states(C.byref(desc.desc), n, ptr(np.ascontiguousarray(root, np.float32)),
                                   ptr(np.ascontiguousarray(dof, np.float32)), ptr(out))
    return out

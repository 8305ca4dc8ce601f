"""ctypes binding of libtgsim.so (the in-tree HIP library).

There is no CPU fallback: if the library or its gfx950 code objects are
missing, ``lib()`` raises -- the product path never routes through the oracle."""
from __future__ import annotations

import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TG_LIB_PATH") or os.path.join(HERE, "libtgsim.so")

_lib = None

# (name, argtypes) -- every symbol declared in include/tgsim.h, tg_gogoro.h, tg_walk.h, tg_gogoro_paper.h
_VP = C.c_void_p
SIGNATURES = {
    "tg_sim_create": [C.POINTER(abi.tg_model_desc), C.POINTER(abi.tg_sim_params), C.c_int32, C.c_int32,
                      C.POINTER(C.c_void_p)],
    "tg_sim_destroy": [_VP],
    "tg_set_stream": [_VP, _VP],
    "tg_state_ptrs": [_VP, C.POINTER(abi.tg_state_view)],
    "tg_bind_state": [_VP, C.POINTER(abi.tg_state_view)],
    "tg_refresh": [_VP],
    "tg_set_dof_position_targets": [_VP, _VP],
    "tg_set_dof_velocity_targets": [_VP, _VP],
    "tg_set_dof_actuation_forces": [_VP, _VP],
    "tg_set_actor_root_state_indexed": [_VP, _VP, _VP, C.c_int32],
    "tg_set_dof_state_indexed": [_VP, _VP, _VP, C.c_int32],
    "tg_set_dof_properties_indexed": [_VP, C.c_int32, _VP, _VP, C.c_int32],
    "tg_set_body_mass_scale_indexed": [_VP, _VP, _VP, C.c_int32],
    "tg_set_shape_friction_indexed": [_VP, _VP, _VP, C.c_int32],
    "tg_set_gravity": [_VP, C.POINTER(C.c_float)],
    "tg_apply_body_forces": [_VP, _VP],
    "tg_apply_rigid_body_force_tensors": [_VP, _VP, _VP, C.c_int32],
    "tg_set_heightfield": [_VP, _VP, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float],
    "tg_simulate": [_VP],
    "tg_get_sim_params": [_VP, C.POINTER(abi.tg_sim_params)],
    "tg_set_sim_params": [_VP, C.POINTER(abi.tg_sim_params)],
    "tg_rigid_body_states": [_VP, _VP],
    "tg_sync": [_VP],
    "tg_philox4x32_10": [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)],
    "tg_rng_fill": [_VP, C.c_int32, C.c_uint64, C.c_uint64, _VP, C.c_int32],
    "tg_debug_fill_lds": [_VP, C.c_uint32],
    "tg_composite": [_VP, _VP, C.c_int32],
    "tg_last_error": [],
    "tg_set_kernel_timing": [_VP, C.c_int32],
    "tg_read_kernel_timing": [_VP, C.POINTER(C.c_double), C.POINTER(C.c_int64)],
    "tg_compiled_model_hashes": [C.POINTER(C.c_uint64), C.c_int32],
    "tg_model_jit": [C.c_uint64, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p],
    # native URDF loading (csrc/model_load.cpp)
    "tg_model_parse": [C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int32, C.c_char_p, C.POINTER(C.c_void_p)],
    "tg_model_load": [C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int32, C.c_char_p, C.c_char_p,
                      C.POINTER(C.c_void_p)],
    "tg_model_get_desc": [C.c_void_p, C.c_void_p],
    "tg_model_dof_name": [C.c_void_p, C.c_int32],
    "tg_model_link_name": [C.c_void_p, C.c_int32],
    "tg_model_dof_limits": [C.c_void_p, C.c_int32, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                            C.POINTER(C.c_float)],
    "tg_model_source": [C.c_void_p],
    "tg_model_last_error": [],
    "tg_model_free": [C.c_void_p],
    "tg_gogoro_step": [_VP, C.POINTER(abi.tg_gogoro_params), C.POINTER(abi.tg_gogoro_buffers), _VP, C.c_int32,
                       _VP, _VP, _VP, _VP, _VP, C.c_uint64, C.c_uint64],
    "tg_gogoro_pre_physics": [_VP, C.POINTER(abi.tg_gogoro_params), C.POINTER(abi.tg_gogoro_buffers), _VP, _VP,
                              C.c_uint64],
    "tg_gogoro_post_physics": [_VP, C.POINTER(abi.tg_gogoro_params), C.POINTER(abi.tg_gogoro_buffers), _VP, _VP,
                               _VP, _VP, C.c_uint64],
    "tg_gogoro_reset_idx": [_VP, C.POINTER(abi.tg_gogoro_params), C.POINTER(abi.tg_gogoro_buffers), _VP,
                            C.c_int32, _VP, C.c_uint64],
    "tg_paper_pre_physics": [_VP, C.POINTER(abi.tg_paper_params), C.POINTER(abi.tg_paper_buffers), _VP, C.c_uint64],
    "tg_paper_post_physics": [_VP, C.POINTER(abi.tg_paper_params), C.POINTER(abi.tg_paper_buffers), _VP, _VP, _VP,
                              _VP, _VP, C.c_uint64],
    "tg_paper_reset_idx": [_VP, C.POINTER(abi.tg_paper_params), C.POINTER(abi.tg_paper_buffers), _VP, C.c_int32,
                           _VP, C.c_uint64],
    "tg_paper_step": [_VP, C.POINTER(abi.tg_paper_params), C.POINTER(abi.tg_paper_buffers), _VP, C.c_int32,
                      C.c_uint64],
    "tg_walk_pre_physics": [_VP, C.POINTER(abi.tg_walk_params), C.POINTER(abi.tg_walk_buffers), _VP],
    "tg_walk_step": [_VP, C.POINTER(abi.tg_walk_params), C.POINTER(abi.tg_walk_buffers), _VP, C.c_int32, _VP, _VP,
                     C.c_uint64],
    "tg_walk_post_physics": [_VP, C.POINTER(abi.tg_walk_params), C.POINTER(abi.tg_walk_buffers), _VP, _VP,
                             C.c_uint64],
    "tg_walk_reset_idx": [_VP, C.POINTER(abi.tg_walk_params), C.POINTER(abi.tg_walk_buffers), _VP, C.c_int32,
                          _VP, C.c_uint64],
}


RESTYPES = {"tg_last_error": C.c_char_p, "tg_compiled_model_hashes": C.c_uint64, "tg_philox4x32_10": None,
            "tg_model_dof_name": C.c_char_p, "tg_model_link_name": C.c_char_p, "tg_model_source": C.c_char_p,
            "tg_model_last_error": C.c_char_p, "tg_model_free": None}


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                               "g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = RESTYPES.get(name, C.c_int)
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().tg_last_error().decode(errors="replace")
        raise RuntimeError(f"tgsim {what} failed ({rc}): {msg}")


def compiled_hashes():
    n = lib().tg_compiled_model_hashes(None, 0)
    arr = (C.c_uint64 * max(int(n), 1))()
    lib().tg_compiled_model_hashes(arr, int(n))
    return [int(arr[i]) for i in range(int(n))]

"""Python face of one libtgsim simulation: the part of ``gymapi.Gym`` the
reference tasks use (create_sim/load_asset/create_actor, the tensor API,
simulate), with torch tensors as zero-copy state views.

Reference calls mirrored (isaacgymenvs/tasks/...):
  acquire_actor_root_state_tensor / acquire_dof_state_tensor + wrap_tensor
      -> Sim.root_state [N,13], Sim.dof_state [N*D,2]      (gogoro_new.py:125-130)
  refresh_*_tensor -> Sim.refresh() (state is live: nothing copied; REQUIRED after writes
      through the dof_props / env_dirty views, which take effect at the next simulate only
      after it -- the library skips the compose launch while no env can be dirty)  (gogoro_new.py:141-142)
  set_dof_position/velocity_target_tensor -> Sim.set_dof_*_targets (gogoro_new.py:364,369)
  set_actor_root_state_tensor_indexed / set_dof_state_tensor_indexed  (gogoro_new.py:547,552)
  set_actor_dof_properties (per env)   -> Sim.set_dof_properties_indexed (gogoro_new.py:294,601)
  simulate / fetch_results             -> Sim.simulate / Sim.sync (vec_task.py:335,339)
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np
import torch

from . import abi
from ._lib import check, lib
from .model.urdf import Model

HERE = os.path.dirname(os.path.abspath(__file__))
COMPILED = os.path.join(HERE, "model", "compiled")


def load_model(name: str) -> Model:
    with open(os.path.join(COMPILED, f"{name}.json")) as f:
        return Model.from_json(f.read())


def load_asset(path: str, name: str | None = None, locked=(), extra_shapes=(), mesh_root: str | None = None,
               shape_friction: dict | None = None) -> Model:
    """gym.load_asset of a URDF at run time (the reference: tasks/gogoro_new.py:198-213):
    parse the file, merge fixed and ``locked`` joints into rigid groups.  A
    ``Sim`` over a model that is not compiled into libtgsim.so compiles its
    kernels on first use (``ensure_specialisation``), so any URDF runs without
    a library rebuild."""
    from .model.urdf import load_urdf
    m = load_urdf(path, name or os.path.splitext(os.path.basename(path))[0], mesh_root=mesh_root,
                  extra_shapes=list(extra_shapes), shape_friction=shape_friction)
    m.build_groups(list(locked))
    return m


def jit_cache_dir() -> str:
    """Where run-time specialisations are cached (TG_JIT_CACHE, default
    ~/.cache/thormang_isaacgym_amd/jit)."""
    d = os.environ.get("TG_JIT_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "thormang_isaacgym_amd",
                                                        "jit")
    os.makedirs(d, exist_ok=True)
    return d


def compiled_model_hashes() -> set:
    n = int(lib().tg_compiled_model_hashes(None, 0))
    arr = (C.c_uint64 * max(n, 1))()
    lib().tg_compiled_model_hashes(arr, n)
    return {int(arr[i]) for i in range(n)}


def ensure_specialisation(model: Model, desc: abi.ModelDesc | None = None) -> bool:
    """Make sure libtgsim can step ``model``: a no-op for a compiled-in model;
    otherwise the model's constexpr tables (model/codegen.py) are compiled by
    hipRTC for gfx950 inside the library (tg_model_jit, cached on disk by hash)
    and registered.  Returns True when a run-time specialisation is used."""
    from .model import codegen
    desc = desc or abi.ModelDesc(model)
    if desc.hash in compiled_model_hashes():
        return False
    cname = "Model_jit_%016x" % desc.hash
    src = codegen.emit(model, cname)
    check(lib().tg_model_jit(C.c_uint64(desc.hash), cname.encode(), src.encode(), None, jit_cache_dir().encode()),
          "tg_model_jit (run-time load_asset)")
    return True


class NativeModel:
    """gym.load_asset through the C ABI alone (tg_model_load, csrc/model_load.cpp):
    the library parses the URDF, builds the tg_model_desc and the
    specialisation's traits and (``jit=True``) compiles them with hipRTC -- what
    a caller without Python gets; ``Sim`` accepts it in place of a ``Model``.
    The descriptor arrays live in the library until the object is freed."""

    def __init__(self, path: str, locked=(), mesh_root: str | None = None, name: str | None = None,
                 jit: bool = True):
        L = lib()
        h = C.c_void_p()
        names = (C.c_char_p * max(len(locked), 1))(*[n.encode() for n in locked])
        args = [path.encode(), name.encode() if name else None, names, len(locked),
                mesh_root.encode() if mesh_root else None]
        rc = L.tg_model_load(*args, jit_cache_dir().encode(), C.byref(h)) if jit else \
            L.tg_model_parse(*args, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"tg_model_load({path}): {L.tg_model_last_error().decode()} (rc {rc})")
        self._h = h
        self.desc = abi.tg_model_desc()
        check(L.tg_model_get_desc(h, C.byref(self.desc)), "tg_model_get_desc")
        self.hash = int(self.desc.model_hash)
        self.num_bodies, self.num_dof = self.desc.num_links, self.desc.num_dofs
        self.num_groups, self.num_shapes = self.desc.num_groups, self.desc.num_shapes
        self.dof_names = [L.tg_model_dof_name(h, i).decode() for i in range(self.num_dof)]
        self.link_names = [L.tg_model_link_name(h, i).decode() for i in range(self.num_bodies)]
        S = self.num_shapes
        self.arrays = {"shape_friction": np.ctypeslib.as_array(self.desc.shape_friction, (S,)).astype(np.float32)
                       if S else np.zeros(0, np.float32)}
        self.jit = jit and self.hash not in compiled_model_hashes()

    def source(self) -> str:
        return lib().tg_model_source(self._h).decode()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().tg_model_free(self._h)
            self._h = None


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


class Sim:
    def __init__(self, model: Model, params: abi.tg_sim_params, num_envs: int, device: str = "cuda:0",
                 jit_hash: int | None = None):
        """``jit_hash`` (test hook): register the model under this hash instead
        of its own, so even a compiled-in model runs on a run-time
        (tg_model_jit) specialisation -- the JIT path can then be compared
        with the compiled one on identical inputs."""
        if not device.startswith("cuda"):
            raise RuntimeError(f"libtgsim runs on an MI355X ('cuda:N' device), got {device!r}; "
                               "there is no CPU physics path outside the test oracle")
        self.device = torch.device(device)
        self.model = model
        self.num_envs = N = int(num_envs)
        self.params = params
        torch.cuda.set_device(self.device)
        if isinstance(model, NativeModel):   # loaded (and compiled) by the library itself
            self.desc = model
            self.D, self.G, self.L, self.S = model.num_dof, model.num_groups, model.num_bodies, model.num_shapes
            self.jit = model.jit
        else:
            self.desc = abi.ModelDesc(model)
            if jit_hash is not None:
                self.desc.hash = int(jit_hash)
                self.desc.desc.model_hash = int(jit_hash)
            self.D, self.G, self.L, self.S = model.num_dof, model.num_groups, model.num_bodies, len(model.shapes)
            self.jit = ensure_specialisation(model, self.desc)
        h = C.c_void_p()
        check(lib().tg_sim_create(C.byref(self.desc.desc), C.byref(params), N, self.device.index or 0, C.byref(h)),
              "tg_sim_create")
        self._h = h
        self.stream = torch.cuda.current_stream(self.device)
        check(lib().tg_set_stream(self._h, C.c_void_p(self.stream.cuda_stream)), "tg_set_stream")
        f32 = dict(dtype=torch.float32, device=self.device)
        D, G = self.D, self.G
        self.root_state = torch.zeros(N, 13, **f32)
        self.dof_state = torch.zeros(N * D, 2, **f32)
        self.dof_pos_target = torch.zeros(N, D, **f32)
        self.dof_vel_target = torch.zeros(N, D, **f32)
        self.dof_actuation = torch.zeros(N, D, **f32)
        self.dof_props = torch.zeros(abi.TG_NUM_PROPS, N, D, **f32)
        self.body_force = torch.zeros(N, G, 6, **f32)
        self.env_origin = torch.zeros(N, 3, **f32)
        self.env_dirty = torch.zeros(N, dtype=torch.uint8, device=self.device)
        v = abi.tg_state_view()
        for k in ("root_state", "dof_state", "dof_pos_target", "dof_vel_target", "dof_actuation", "dof_props",
                  "body_force", "env_origin", "env_dirty"):
            setattr(v, k, getattr(self, k).data_ptr())
        check(lib().tg_bind_state(self._h, C.byref(v)), "tg_bind_state")
        self.all_ids = torch.arange(N, dtype=torch.int32, device=self.device)
        # mirrors of the per-env properties the library holds (read back by
        # get_* style inspection and the parity harness; never on the hot path)
        self.body_mass_scale = torch.ones(N, self.L, **f32)
        self.shape_friction = torch.as_tensor(np.asarray(self.desc.arrays["shape_friction"], np.float32),
                                              device=self.device).repeat(N, 1)
        self.gravity = [float(x) for x in params.gravity]

    @property
    def handle(self):
        return self._h

    # ---------------------------------------------------------------- tensor API
    def refresh(self):
        """refresh_*_tensor: the views are live, nothing is copied.  Call it after
        writing through ``dof_props`` / ``env_dirty`` (tg_refresh re-arms the
        compose launch those writes need)."""
        check(lib().tg_refresh(self._h), "refresh")

    def set_dof_position_targets(self, t: torch.Tensor):
        check(lib().tg_set_dof_position_targets(self._h, _ptr(self._dev(t))), "set_dof_position_target_tensor")

    def set_dof_velocity_targets(self, t: torch.Tensor):
        check(lib().tg_set_dof_velocity_targets(self._h, _ptr(self._dev(t))), "set_dof_velocity_target_tensor")

    def set_dof_actuation_forces(self, t: torch.Tensor):
        check(lib().tg_set_dof_actuation_forces(self._h, _ptr(self._dev(t))), "set_dof_actuation_force_tensor")

    def set_actor_root_state_indexed(self, root: torch.Tensor, ids: torch.Tensor):
        ids = self._ids(ids)
        check(lib().tg_set_actor_root_state_indexed(self._h, _ptr(self._dev(root)), _ptr(ids), ids.numel()),
              "set_actor_root_state_tensor_indexed")
        return True

    def set_dof_state_indexed(self, dof: torch.Tensor, ids: torch.Tensor):
        ids = self._ids(ids)
        check(lib().tg_set_dof_state_indexed(self._h, _ptr(self._dev(dof)), _ptr(ids), ids.numel()),
              "set_dof_state_tensor_indexed")
        return True

    def set_dof_properties_indexed(self, field: int, vals: torch.Tensor, ids: torch.Tensor):
        ids = self._ids(ids)
        check(lib().tg_set_dof_properties_indexed(self._h, int(field), _ptr(self._dev(vals)), _ptr(ids),
                                                  ids.numel()), "set_actor_dof_properties")

    def set_body_mass_scale_indexed(self, scale: torch.Tensor, ids: torch.Tensor):
        ids = self._ids(ids)
        check(lib().tg_set_body_mass_scale_indexed(self._h, _ptr(self._dev(scale)), _ptr(ids), ids.numel()),
              "mass scale")
        # host-side mirror of the rigid-body mass properties (get_actor_rigid_body_properties)
        self.body_mass_scale[ids.long()] = scale[ids.long()]

    def set_shape_friction_indexed(self, mu: torch.Tensor, ids: torch.Tensor):
        ids = self._ids(ids)
        check(lib().tg_set_shape_friction_indexed(self._h, _ptr(self._dev(mu)), _ptr(ids), ids.numel()), "friction")
        self.shape_friction[ids.long()] = mu[ids.long()]   # mirror (get_actor_rigid_shape_properties)

    def set_gravity(self, g):
        arr = (C.c_float * 3)(*[float(x) for x in g])
        check(lib().tg_set_gravity(self._h, arr), "set_gravity")
        self.gravity = [float(x) for x in g]

    def apply_body_forces(self, wrench: torch.Tensor):
        """Group wrenches [N, G, 6] (world force, torque about the group com) for the next simulate."""
        check(lib().tg_apply_body_forces(self._h, _ptr(self._dev(wrench))), "apply_body_forces")

    ENV_SPACE, LOCAL_SPACE = 0, 1

    def apply_rigid_body_force_tensors(self, forces, torques=None, space: int = 0):
        """gym.apply_rigid_body_force_tensors(sim, forceTensor, torqueTensor, space)
        (tasks/gogoro_realistic_turning_sim_paper.py:457): forces / torques
        [N*L, 3] (or [N, L, 3]) at the rigid bodies' coms, world (ENV_SPACE) or
        body frame (LOCAL_SPACE), for the next simulate.  Returns True, as gym does."""
        def flat(t):
            if t is None:
                return None
            t = self._dev(t)
            if t.numel() != self.num_envs * self.L * 3:
                raise ValueError(f"rigid-body force tensor must hold N*L*3 = {self.num_envs * self.L * 3} floats, "
                                 f"got shape {tuple(t.shape)}")
            return t.reshape(-1, 3).contiguous()
        f, t = flat(forces), flat(torques)
        check(lib().tg_apply_rigid_body_force_tensors(self._h, _ptr(f), _ptr(t), int(space)),
              "apply_rigid_body_force_tensors")
        self._keep_forces = (f, t)   # the reduction runs on the sim stream; hold the inputs until the next call
        return True

    def set_heightfield(self, heights, horizontal_scale: float = 1.0, vertical_scale: float = 1.0,
                        origin_x: float = 0.0, origin_y: float = 0.0, friction: float = 1.0):
        """gym.add_triangle_mesh of a heightfield trimesh (see tg_set_heightfield); None = flat plane."""
        if heights is None:
            check(lib().tg_set_heightfield(self._h, None, 0, 0, 1.0, 1.0, 0.0, 0.0, 1.0), "set_heightfield")
            return
        if isinstance(heights, torch.Tensor):
            heights = heights.detach().cpu().numpy()
        h = np.ascontiguousarray(np.asarray(heights, np.float32))
        if h.ndim != 2:
            raise ValueError(f"heightfield must be [rows, cols], got shape {h.shape}")
        check(lib().tg_set_heightfield(self._h, h.ctypes.data_as(C.c_void_p), h.shape[0], h.shape[1],
                                       float(horizontal_scale), float(vertical_scale), float(origin_x),
                                       float(origin_y), float(friction)), "set_heightfield")

    def simulate(self):
        check(lib().tg_simulate(self._h), "simulate")

    def debug_fill_lds(self, pattern: int = 0x7FC00000):
        """tg_debug_fill_lds: every CU's LDS filled with ``pattern`` (default a
        quiet NaN) on this sim's stream -- the stale-LDS tests' probe."""
        check(lib().tg_debug_fill_lds(self._h, C.c_uint32(pattern)), "debug_fill_lds")

    def get_sim_params(self) -> abi.tg_sim_params:
        """gym.get_sim_params (vec_task.py:650): a copy of the live params."""
        sp = abi.tg_sim_params()
        check(lib().tg_get_sim_params(self._h, C.byref(sp)), "get_sim_params")
        return sp

    def set_sim_params(self, sp: abi.tg_sim_params):
        """gym.set_sim_params (vec_task.py:660), effective from the next simulate
        (substeps 0: simulate passes the state through, the recorded-physics replays)."""
        check(lib().tg_set_sim_params(self._h, C.byref(sp)), "set_sim_params")
        self.params = sp
        self.gravity = [float(x) for x in sp.gravity]

    def acquire_rigid_body_state_tensor(self) -> torch.Tensor:
        """gym.acquire_rigid_body_state_tensor: [N*L, 13] world link states
        (origin pos, quat xyzw, com linvel, angvel), links in model order;
        filled by refresh_rigid_body_state_tensor."""
        if getattr(self, "rigid_body_state", None) is None:
            self.rigid_body_state = torch.zeros(self.num_envs * self.L, 13, dtype=torch.float32, device=self.device)
        return self.rigid_body_state

    def refresh_rigid_body_state_tensor(self):
        rb = self.acquire_rigid_body_state_tensor()
        check(lib().tg_rigid_body_states(self._h, _ptr(rb)), "refresh_rigid_body_state_tensor")

    def sync(self):
        check(lib().tg_sync(self._h), "sync")

    def set_kernel_timing(self, period: int):
        """Bracket every ``period``-th articulation step kernel launch with HIP
        events on the sim stream (``True``/1: every launch, 0/``False``: off);
        a negative period -W brackets windows of W consecutive step-kernel
        launches with one event pair (a window another launch of the library
        falls into is dropped)."""
        check(lib().tg_set_kernel_timing(self._h, int(period)), "set_kernel_timing")

    def read_kernel_timing(self):
        """(total kernel ms, launches) since the last read; waits for the recorded launches."""
        ms, n = C.c_double(), C.c_int64()
        check(lib().tg_read_kernel_timing(self._h, C.byref(ms), C.byref(n)), "read_kernel_timing")
        return ms.value, n.value

    def close(self):
        if getattr(self, "_h", None):
            lib().tg_sim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- helpers
    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"expected a contiguous float32 tensor on {self.device}, got {t.dtype} on {t.device}")
        return t

    def _ids(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(device=self.device, dtype=torch.int32).contiguous()
        return ids

    def props_view(self, field: int) -> torch.Tensor:
        """[N,D] live view of one per-env DOF property field (tgsim.h TG_PROP_*)."""
        return self.dof_props[field]

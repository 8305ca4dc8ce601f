"""C-ABI checks that need no GPU: the library loads, exports every symbol the
public headers declare, rejects bad arguments with a message, and the ctypes
struct layouts match the C headers."""
import ctypes as C
import os
import re
import subprocess

import pytest

from thormang_isaacgym_amd import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    out = set()
    for h in ("tgsim.h", "tg_gogoro.h", "tg_walk.h", "tg_gogoro_paper.h"):
        text = open(os.path.join(REPO, "include", h)).read()
        out |= set(re.findall(r"^(?:int|void|const char \*|uint64_t)\s*(tg_\w+)\(", text, re.M))
    return out


def test_headers_declare_expected_entry_points():
    syms = declared_symbols()
    for s in ("tg_sim_create", "tg_simulate", "tg_set_actor_root_state_indexed", "tg_gogoro_post_physics",
              "tg_last_error", "tg_bind_state"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from thormang_isaacgym_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libtgsim.so not built")
    L = _lib.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == declared_symbols()


def test_compiled_specialisations_match_models():
    from thormang_isaacgym_amd import _lib
    from thormang_isaacgym_amd.model.codegen import model_registry
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libtgsim.so not built")
    hashes = set(_lib.compiled_hashes())
    for _, m in model_registry():
        assert abi.ModelDesc(m).hash in hashes, m.name


def test_create_rejects_unknown_model_without_gpu():
    from thormang_isaacgym_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libtgsim.so not built")
    from tests.physics_models import pendulum
    d = abi.ModelDesc(pendulum(l=0.123))   # not compiled in
    d.desc.model_hash = 1
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1}, {}, 1)
    h = C.c_void_p()
    rc = _lib.lib().tg_sim_create(C.byref(d.desc), C.byref(sp), 1, 0, C.byref(h))
    assert rc != 0
    assert b"no specialisation" in _lib.lib().tg_last_error()


def test_jit_compiles_a_model_that_is_not_compiled_in(tmp_path):
    """tg_model_jit (gym.load_asset at run time): hipRTC compiles the
    articulation kernels for a URDF that is not among the compiled-in models
    and caches the gfx950 code object.  Without a GPU the module load that
    follows fails -- the cached object shows the compile went through."""
    from thormang_isaacgym_amd import _lib
    from thormang_isaacgym_amd.model import codegen
    from tests.test_gpu_physics import jit_walker
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libtgsim.so not built")
    m = jit_walker()
    d = abi.ModelDesc(m)
    assert d.hash not in set(_lib.compiled_hashes())
    cname = "Model_jit_%016x" % d.hash
    rc = _lib.lib().tg_model_jit(C.c_uint64(d.hash), cname.encode(), codegen.emit(m, cname).encode(), None,
                                 str(tmp_path).encode())
    files = os.listdir(tmp_path)
    assert any(f.startswith("tgjit_%016x_" % d.hash) and f.endswith(".co") for f in files), \
        (files, _lib.lib().tg_last_error())
    if rc != 0:   # no GPU here: only the load may fail
        assert b"loading the run-time code object" in _lib.lib().tg_last_error()


def test_struct_layouts_match_c():
    """Compile a tiny C program printing sizeof/offsetof and compare with ctypes."""
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "tg_gogoro.h"
#include "tg_walk.h"
#include "tg_gogoro_paper.h"
int main(void){
 printf("%zu %zu %zu %zu %zu\n", sizeof(tg_model_desc), sizeof(tg_sim_params), sizeof(tg_state_view),
        sizeof(tg_gogoro_params), sizeof(tg_gogoro_buffers));
 printf("%zu %zu %zu %zu %zu\n", offsetof(tg_gogoro_params, max_episode_length), offsetof(tg_gogoro_params, seed),
        offsetof(tg_model_desc, model_hash), sizeof(tg_walk_params), sizeof(tg_walk_buffers));
 printf("%zu %zu %zu %zu\n", sizeof(tg_paper_params), offsetof(tg_paper_params, head_com),
        offsetof(tg_paper_params, seed), sizeof(tg_paper_buffers));
 return 0;}
'''
    tmp = os.path.join(REPO, "oracle", "_build")
    os.makedirs(tmp, exist_ok=True)
    c = os.path.join(tmp, "layout.c")
    exe = os.path.join(tmp, "layout")
    open(c, "w").write(src)
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    sizes = [C.sizeof(t) for t in (abi.tg_model_desc, abi.tg_sim_params, abi.tg_state_view, abi.tg_gogoro_params,
                                   abi.tg_gogoro_buffers)]
    offs = [abi.tg_gogoro_params.max_episode_length.offset, abi.tg_gogoro_params.seed.offset,
            abi.tg_model_desc.model_hash.offset, C.sizeof(abi.tg_walk_params), C.sizeof(abi.tg_walk_buffers)]
    paper = [C.sizeof(abi.tg_paper_params), abi.tg_paper_params.head_com.offset, abi.tg_paper_params.seed.offset,
             C.sizeof(abi.tg_paper_buffers)]
    assert [int(x) for x in out] == sizes + offs + paper

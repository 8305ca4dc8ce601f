"""Native URDF loading (tg_model_parse, csrc/model_load.cpp) against the Python
host's loader (model/urdf.py load_urdf + build_groups, abi.model_arrays /
model_hash, model/codegen.py emit): the same tg_model_desc arrays, hash and
constexpr traits text -- gym.load_asset (/root/reference/isaacgymenvs/tasks/
gogoro_new.py:198-213) for a caller without Python.  CPU only: parsing needs
no device (tg_model_load's hipRTC step is covered by the GPU test)."""
import ctypes as C
import os

import numpy as np
import pytest

from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd._lib import lib
from thormang_isaacgym_amd.model import codegen
from thormang_isaacgym_amd.model.urdf import load_urdf

HERE = os.path.dirname(os.path.abspath(__file__))
URDF = os.path.join(HERE, "golden", "urdf", "loader_tree.urdf")
MESHES = os.path.join(HERE, "golden", "urdf")
REF = "/root/reference/assets/urdf/gogoro"
TG_ERR_MODEL = -3   # include/tgsim.h

ARRAYS = [("link_parent", "num_links", 1, np.int32), ("link_group", "num_links", 1, np.int32),
          ("link_dof", "num_links", 1, np.int32), ("link_jtype", "num_links", 1, np.int32),
          ("link_origin", "num_links", 12, np.float32), ("link_axis", "num_links", 3, np.float32),
          ("link_inertia", "num_links", 10, np.float32), ("group_root", "num_groups", 1, np.int32),
          ("group_parent", "num_groups", 1, np.int32), ("dof_locked", "num_dofs", 1, np.int32),
          ("shape_link", "num_shapes", 1, np.int32), ("shape_kind", "num_shapes", 1, np.int32),
          ("shape_pose", "num_shapes", 12, np.float32), ("shape_params", "num_shapes", 4, np.float32),
          ("shape_friction", "num_shapes", 1, np.float32)]


def native(path, locked=(), mesh_root=None, name=None):
    L = lib()
    h = C.c_void_p()
    names = (C.c_char_p * max(len(locked), 1))(*[n.encode() for n in locked])
    rc = L.tg_model_parse(path.encode(), name.encode() if name else None, names, len(locked),
                          mesh_root.encode() if mesh_root else None, C.byref(h))
    assert rc == 0, L.tg_model_last_error().decode()
    d = abi.tg_model_desc()
    assert L.tg_model_get_desc(h, C.byref(d)) == 0
    out = {}
    for k, nk, w, dt in ARRAYS:
        n = getattr(d, nk) * w
        ptr = getattr(d, k)
        out[k] = np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)
    info = dict(hash=int(d.model_hash), source=L.tg_model_source(h).decode(),
                dofs=[L.tg_model_dof_name(h, i).decode() for i in range(d.num_dofs)],
                links=[L.tg_model_link_name(h, i).decode() for i in range(d.num_links)],
                limits=[], counts=(d.num_links, d.num_dofs, d.num_groups, d.num_shapes))
    for i in range(d.num_dofs):
        v = [C.c_float() for _ in range(4)]
        assert L.tg_model_dof_limits(h, i, *[C.byref(x) for x in v]) == 0
        info["limits"].append([x.value for x in v])
    L.tg_model_free(h)
    return out, info


def python_side(path, locked=(), mesh_root=None, name=None):
    m = load_urdf(path, name or os.path.splitext(os.path.basename(path))[0], mesh_root=mesh_root)
    m.build_groups(list(locked))
    d = abi.ModelDesc(m)
    return m, d


def compare(path, locked=(), mesh_root=None, name=None, exact_hash=True):
    a, info = native(path, locked, mesh_root, name)
    m, d = python_side(path, locked, mesh_root, name)
    assert info["counts"] == (m.num_bodies, m.num_dof, m.num_groups, len(m.shapes))
    assert info["dofs"] == m.dof_names
    assert info["links"] == [l.name for l in m.links]
    for k, _, _, _ in ARRAYS:
        ref = np.ascontiguousarray(d.arrays[k]).reshape(-1)
        if ref.dtype == np.int32:
            np.testing.assert_array_equal(a[k], ref, err_msg=k)
        else:
            np.testing.assert_allclose(a[k], ref, rtol=0, atol=1e-6, err_msg=k)
    props = abi.default_dof_props(m, 1)[:, 0, :]
    lim = np.array(info["limits"], np.float32).reshape(-1, 4)
    if len(lim):
        for c, p in enumerate((abi.TG_PROP_LOWER, abi.TG_PROP_UPPER, abi.TG_PROP_EFFORT, abi.TG_PROP_VELOCITY)):
            np.testing.assert_allclose(lim[:, c], props[p], rtol=1e-7)
    if exact_hash:
        assert info["hash"] == d.hash
        cname = "Model_jit_%016x" % d.hash
        assert info["source"] == codegen.emit(m, cname)
    return info, m, d


def test_native_loader_matches_the_python_host_on_every_joint_and_shape_kind():
    info, m, d = compare(URDF, locked=["j_seat"], mesh_root=MESHES)
    # the asset covers what it should: every joint type, a lock, all shape kinds
    assert sorted(set(j.jtype for j in m.joints)) == [0, 1, 2]
    assert sorted(set(abi.SHAPE_KIND[s.kind] for s in m.shapes)) == [0, 1, 2]
    assert m.locked_dofs and m.num_groups < m.num_bodies
    # fitted tyre: crown 0.25 exactly, the minor radius from the coarse mesh's shoulder band
    tor = [s for s in m.shapes if s.kind == "torus"][0]
    assert abs(tor.params[0] + tor.params[1] - 0.25) < 1e-3 and abs(tor.params[1] - 0.05) < 0.015


def test_native_loader_without_locks_or_meshes():
    compare(URDF)


def test_native_loader_reports_errors():
    L = lib()
    h = C.c_void_p()
    names = (C.c_char_p * 1)(b"no_such_joint")
    assert L.tg_model_parse(URDF.encode(), None, names, 1, None, C.byref(h)) != 0
    assert b"no_such_joint" in L.tg_model_last_error()
    assert L.tg_model_parse(b"/nonexistent.urdf", None, None, 0, None, C.byref(h)) != 0
    assert b"not found" in L.tg_model_last_error()
    bad = os.path.join(HERE, "golden", "urdf", "tyre.obj")   # not XML
    assert L.tg_model_parse(bad.encode(), None, None, 0, None, C.byref(h)) != 0


MINI = """<robot name="r">
  <link name="R"><inertial><mass value="{m}"/><inertia ixx="1" ixy="0" ixz="0" iyy="1" iyz="0" izz="1"/></inertial></link>
  <link name="B"/><link name="C"/>
  <joint name="rb" type="revolute"><parent link="R"/><child link="B"/><limit effort="1" velocity="1" lower="-1" upper="1"/></joint>
  {extra}
</robot>"""


def _parse_text(tmp_path, text):
    p = tmp_path / "m.urdf"
    p.write_text(text)
    L = lib()
    h = C.c_void_p()
    rc = L.tg_model_parse(str(p).encode(), None, None, 0, None, C.byref(h))
    if rc == 0:
        L.tg_model_free(h)
    return rc, L.tg_model_last_error().decode()


def test_native_loader_rejects_malformed_urdfs(tmp_path):
    """a joint cycle (R->B, B->C, C->B), a link with two parent
    joints, a malformed number and runaway element nesting each return
    TG_ERR_MODEL with a message, instead of overflowing the stack or reading
    the value as 0 as strtod did."""
    ok = '<joint name="bc" type="fixed"><parent link="B"/><child link="C"/></joint>'
    assert _parse_text(tmp_path, MINI.format(m="1.5", extra=ok))[0] == 0
    cyc = ok + '<joint name="cb" type="fixed"><parent link="C"/><child link="B"/></joint>'
    rc, msg = _parse_text(tmp_path, MINI.format(m="1.5", extra=cyc))
    assert rc == TG_ERR_MODEL and "more than one joint" in msg, msg
    rc, msg = _parse_text(tmp_path, MINI.format(m="1.5kg", extra=ok))
    assert rc == TG_ERR_MODEL and "malformed number" in msg and "1.5kg" in msg, msg
    rc, msg = _parse_text(tmp_path, MINI.format(m="", extra=ok))
    assert rc == TG_ERR_MODEL and "malformed number" in msg, msg
    deep = "<a>" * 5000 + "</a>" * 5000
    rc, msg = _parse_text(tmp_path, MINI.format(m="1", extra=deep))
    assert rc == TG_ERR_MODEL and "nested deeper" in msg, msg


def test_native_loader_number_parsing_ignores_the_host_locale(tmp_path):
    """A C / JNI host that set LC_NUMERIC to a comma-decimal locale still gets
    0.5 for "0.5" (the parser reads in the classic locale)."""
    import locale
    ok = '<joint name="bc" type="fixed"><parent link="B"/><child link="C"/></joint>'
    p = tmp_path / "m.urdf"
    p.write_text(MINI.format(m="0.5", extra=ok))
    saved = locale.setlocale(locale.LC_NUMERIC)
    for name in ("de_DE.UTF-8", "de_DE.utf8", "fr_FR.UTF-8", "C"):
        try:
            locale.setlocale(locale.LC_NUMERIC, name)
            break
        except locale.Error:
            continue
    try:
        a, _ = native(str(p))
    finally:
        locale.setlocale(locale.LC_NUMERIC, saved)
    assert abs(a["link_inertia"][0] - 0.5) < 1e-7, a["link_inertia"][:10]


def test_native_loader_parses_numbers_as_python_float(tmp_path):
    """a number attribute reads as the Python host's float() reads
    it (model/urdf.py) -- blanks around it, underscores between digits, an
    exponent, inf / nan in any case -- and what float() rejects (hex floats,
    misplaced underscores, trailing text) is an error."""
    ok = '<joint name="bc" type="fixed"><parent link="B"/><child link="C"/></joint>'
    for text, want in ((" 1_0.5 ", 10.5), ("1E1", 10.0), ("+2.5e-1", 0.25)):
        p = tmp_path / "m.urdf"
        p.write_text(MINI.format(m=text, extra=ok))
        a, _ = native(str(p))
        assert abs(a["link_inertia"][0] - want) < 1e-12 * max(1.0, want), (text, a["link_inertia"][0])
    for text in ("inf", "-Infinity", "NaN", "1e999"):   # accepted by float(); the parse itself must not fail
        rc, msg = _parse_text(tmp_path, MINI.format(m=text, extra=ok))
        assert "malformed number" not in msg, (text, msg)
    for text in ("0x1p3", "1__0", "_1", "1_", "1.5 2", "nan1", "nan(123)", "NAN()"):   # strtod takes nan(...)
        rc, msg = _parse_text(tmp_path, MINI.format(m=text, extra=ok))
        assert rc == TG_ERR_MODEL and "malformed number" in msg, (text, msg)


def test_native_loader_bounds_the_link_chain_depth(tmp_path):
    """the depth-first walk over the joint tree is recursive, so a
    hostile 2000-link chain is refused with a message (no stack exhaustion);
    a 200-link chain still loads."""
    def chain(n):
        links = "".join(f'<link name="L{i}"/>' for i in range(n))
        joints = "".join(f'<joint name="j{i}" type="fixed"><parent link="L{i}"/><child link="L{i + 1}"/></joint>'
                         for i in range(n - 1))
        return f'<robot name="c">{links}{joints}</robot>'
    rc, msg = _parse_text(tmp_path, chain(2000))
    assert rc == TG_ERR_MODEL and "deeper than" in msg, msg
    rc, msg = _parse_text(tmp_path, chain(200))
    assert rc == 0, msg


@pytest.mark.skipif(not os.path.exists(REF), reason="reference assets not present (build container only)")
def test_native_loader_on_the_reference_assets():
    """The registered task's scooter with the reference's locked joints and the
    tyre meshes (model/build_models.py), and the stand-alone Thormang URDF:
    bit-identical arrays, hash and traits text.  (Named apart from the
    compiled-in "gogoro", whose traits carry the fused task epilogue a
    run-time model does not get.)"""
    from thormang_isaacgym_amd.model.build_models import GOGORO_LOCKED
    compare(f"{REF}/urdf/scooter_V13.urdf", locked=GOGORO_LOCKED, mesh_root=f"{REF}/meshes", name="scooter_v13")
    compare(f"{REF}/urdf/thormang3.urdf", name="thormang_urdf")

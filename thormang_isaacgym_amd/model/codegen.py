"""Emit constexpr model traits for the specialised HIP step kernel.

For every compiled model the kernels ``tg::step_par_kernel<M>`` and
``tg::compose_kernel<M>`` (csrc/step_par.h, csrc/articulation.hip) are
instantiated with a traits struct of compile-time tables: the joint tree, the
contact shapes, the lane schedule of the tree-parallel step (``sched``: groups
per step and lane, parents first) and the root->contact-group paths used by
the path-restricted Delassus build.  The model hash
ties a runtime ``tg_model_desc`` to its specialisation (abi.model_hash)."""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from thormang_isaacgym_amd.abi import ModelDesc  # noqa: E402
from thormang_isaacgym_amd.model.urdf import Model  # noqa: E402

BOX_NORMALS = 4   # a box contributes the 4 corners of its lowest face


def _f(x):
    s = f"{float(x):.9g}"
    if "." not in s and "e" not in s:
        s += ".0"
    return s + "f"


def _arr(vals, fmt=str):
    return "{" + ", ".join(fmt(v) for v in vals) + "}"


def shape_rows(kind: int) -> int:
    return BOX_NORMALS if kind == 1 else 1


LANES_PER_ENV = 8   # schedule lanes per env of the tree-parallel step kernel (csrc/step_par.h)
# trees with at least this many groups run on lane pairs (16 lanes per env)
PAIR_MIN_GROUPS = int(os.environ.get("TG_PAIR_MIN_GROUPS", "2"))


def lane_schedule(parent, lanes):
    """Greedy list schedule of the non-root groups onto ``lanes`` lanes.

    Step t holds up to ``lanes`` groups whose parents were all scheduled at an
    earlier step (the root counts as scheduled); groups with the longest path
    to a leaf go first.  Run forward it is a valid top-down order, run in
    reverse a valid bottom-up order (children before parents)."""
    G = len(parent)
    height = [0] * G
    for g in range(G - 1, 0, -1):                 # parents precede children (topological numbering)
        p = parent[g]
        height[p] = max(height[p], height[g] + 1)
    step_of = {0: -1}
    steps = []
    todo = set(range(1, G))
    while todo:
        t = len(steps)
        ready = sorted((g for g in todo if parent[g] in step_of and step_of[parent[g]] < t),
                       key=lambda g: (-height[g], g))
        cur = ready[:lanes]
        for g in cur:
            step_of[g] = t
            todo.discard(g)
        steps.append(cur + [-1] * (lanes - len(cur)))
    return steps or [[-1] * lanes]


def axis_frame(a) -> np.ndarray:
    """Rotation Q (row-major 3x3) whose third column is the unit joint axis ``a``:
    the step kernel works in joint-aligned group frames (v_old = Q v_new), where
    every joint axis is e_z.  Q = I when ``a`` already is e_z."""
    a = np.asarray(a, np.float64)
    a = a / np.linalg.norm(a)
    if np.allclose(a, [0, 0, 1]):
        return np.eye(3)
    ref = np.array([1.0, 0, 0]) if abs(a[0]) < 0.9 else np.array([0, 1.0, 0])
    b1 = np.cross(ref, a)
    b1 /= np.linalg.norm(b1)
    b2 = np.cross(a, b1)
    return np.stack([b1, b2, a], 1)


#: models whose step kernel carries a task's post-physics epilogue (bit 1:
#: ThormangWalk -- selected by tree size in articulation.hip; bit 2: the
#: registered Gogoro task's scooter)
FUSED_GOGORO_MODELS = ("gogoro",)
# models whose task (GogoroPaper) moves the seat locks in place at resets
# (gogoro_paper_task.hip paper_post_kernel<M>): translating locks, link coms kept
PAPER_MODELS = ("gogoro_v12",)


def fused_tasks(m: Model) -> int:
    return (2 if m.name in FUSED_GOGORO_MODELS else 0) | (4 if m.name in PAPER_MODELS else 0)


def translating_locks(m: Model, a: dict) -> dict:
    """The locked prismatic joints inside one rigid group whose windows a fused
    task epilogue moves at every reset (the Gogoro seat offsets base_z ->
    base_x -> base_y, tasks/gogoro_new.py:562-572): moving such a lock only
    translates the links below it, so the epilogue updates the group's
    composite (mass moments) and the placements of the groups hanging below
    instead of re-composing the env (csrc GogoroPost).  Only for models with
    the fused Gogoro epilogue; the joints must form one nested chain in one
    group.  Returns the tables codegen emits (NTL = 0: none)."""
    none = dict(NTL=0, tl_link=[0], tl_dof=[0], tl_group=0, link_tl=[0] * m.num_bodies,
                ag=[], ashape=[], KX=0)
    if not (fused_tasks(m) & 6):
        return none
    L = m.num_bodies
    lpar = [int(x) for x in a["link_parent"]]
    lgrp = [int(x) for x in a["link_group"]]
    groot = set(int(x) for x in a["group_root"])
    tl = [l for l in range(L) if l not in groot and int(a["link_jtype"][l]) == 2 and int(a["link_dof"][l]) >= 0
          and int(a["dof_locked"][int(a["link_dof"][l])])]
    if not tl:
        return none
    assert len(tl) <= 3 and len({lgrp[l] for l in tl}) == 1, "translating locks: one chain of <= 3 in one group"

    def below(l, j):   # link l in the subtree of link j (inclusive)
        while l >= 0:
            if l == j:
                return True
            l = lpar[l]
        return False
    for i in range(1, len(tl)):
        assert below(tl[i], tl[i - 1]), "translating locks must be nested"
    link_tl = [sum(1 << k for k, j in enumerate(tl) if below(l, j)) for l in range(L)]
    gr = [int(x) for x in a["group_root"]]
    ag = [(g, link_tl[lpar[gr[g]]]) for g in range(1, m.num_groups) if link_tl[lpar[gr[g]]]]
    ashape = [(s, link_tl[int(l)]) for s, l in enumerate(a["shape_link"])
              if link_tl[int(l)] and lgrp[int(l)] == lgrp[tl[0]]]
    kx = 10 + 8 * len(tl) + 3 * len(ag) + 3 * len(ashape)
    return dict(NTL=len(tl), tl_link=tl, tl_dof=[int(a["link_dof"][l]) for l in tl], tl_group=lgrp[tl[0]],
                link_tl=link_tl, ag=ag, ashape=ashape, KX=(kx + 3) & ~3)


LDS_BYTES = 160 * 1024


def envs_per_block(G, K, NSA, NCG, MAXD, MAXC, NSTEP, LPE, fused):
    """Envs per workgroup of the step kernel: 16 (every model so far: 4096
    envs = one workgroup per CU), or the largest of 12, 8, 4, 2, 1 whose LDS
    fits when 16 do not (models with many contact rows, e.g. thormang_wb).
    Mirrors csrc/step_par.h ParLayout (the kernel static_asserts the budget)."""
    W = G * 60
    FLG = W + K * K + 8 * K + K + K + 2 * NSA + 12 * NCG + 6 * NCG
    NPW = (NSTEP + 1) // 2
    for epb in (16, 12, 8, 4, 2, 1):
        t_desc = (G * (4 + MAXC) + NCG * MAXD + 3) & ~3
        t_total = t_desc + 4 * NSTEP * LPE + NPW * LPE + 32 + (epb if fused & 4 else 0)
        cb = (FLG + 1 + 3) & ~3
        sepc = (epb * (cb + 32 * G) + t_total) * 4 <= LDS_BYTES
        total = cb + 32 * G if sepc else FLG + 1
        if G <= 8 and G - 1 <= LPE:   # Woodbury slots (ParLayout WOOD; counted whenever it may be on)
            total = ((total + 3) & ~3) + 2 * 8 + 2 * 6 + 2 * 6 * NCG + 2 * max(K, 1) + 4
        es = ((total + 3) & ~3) + (2 if G >= 16 else 0)
        if (epb * es + t_total) * 4 <= LDS_BYTES:
            return epb
    raise ValueError("model does not fit the LDS with one env per workgroup")


def emit(m: Model, cname: str) -> str:
    d = ModelDesc(m)
    a = d.arrays
    G, L, D, S = m.num_groups, m.num_bodies, m.num_dof, len(m.shapes)
    gr = a["group_root"]
    gdof = [int(a["link_dof"][r]) if g > 0 else -1 for g, r in enumerate(gr)]
    gtype = [int(a["link_jtype"][r]) if g > 0 else 0 for g, r in enumerate(gr)]
    gaxis = [a["link_axis"][r] for r in gr]
    gq = [np.eye(3) if g == 0 else axis_frame(gaxis[g]) for g in range(G)]
    sgroup = [int(a["link_group"][l]) for l in a["shape_link"]]
    nrows_n = [shape_rows(int(k)) for k in a["shape_kind"]]
    gpar = [int(x) for x in a["group_parent"]]
    anc = [[0] * G for _ in range(G)]            # anc[k][g] = 1 if g is k or an ancestor of k
    depth = [0] * G
    for k in range(G):
        g = k
        while g >= 0:
            anc[k][g] = 1
            g = gpar[g]
        depth[k] = sum(anc[k]) - 1
    cgroups = sorted(set(sgroup))
    maxd = max([depth[c] for c in cgroups] + [1])
    cpaths = []
    for c in cgroups:                            # root-exclusive path root -> c, topological order
        p = [g for g in range(1, G) if anc[c][g]]
        cpaths.append(p + [0] * (maxd - len(p)))
    shape_cg = [cgroups.index(g) for g in sgroup]
    # 8 schedule lanes x 16 envs per workgroup for every model that fits
    # (envs_per_block): Thormang fills a CU's LDS with 16 envs; for the scooter
    # 8 lanes also beat 2/4 (more Delassus columns in parallel) and 16 envs
    # beat 8 (measured).
    # Every tree with a joint group (PAIR) runs each schedule slot on a lane
    # pair (sub, sub + 8) that splits each group's update: 16 lanes per env, 4
    # wavefronts per workgroup, so 4096 envs put one wavefront on every SIMD
    # (the scooters too since round 3: Gogoro +4 %, GogoroPaper +6 % over 8
    # lanes per env, which left half the SIMDs idle; single-body models keep 8).
    SL = LANES_PER_ENV
    PAIR = 1 if G >= PAIR_MIN_GROUPS else 0
    LPE = SL * (1 + PAIR)
    sched = lane_schedule(gpar, SL)
    children = [[c for c in range(G) if gpar[c] == g] for g in range(G)]
    maxc = max(1, max(len(c) for c in children))
    K = sum(n + (2 if n == 1 else 3) for n in nrows_n)
    EPB = envs_per_block(G, K, max(S, 1), max(len(cgroups), 1), maxd, maxc, len(sched), LPE, fused_tasks(m))
    # compose: link level below its group root (FK level by level), links per group
    lpar = [int(x) for x in a["link_parent"]]
    lgrp = [int(x) for x in a["link_group"]]
    groot = set(int(x) for x in gr)
    level = [0] * L
    for l in range(L):                      # parents precede children
        level[l] = 0 if l in groot else level[lpar[l]] + 1
    # rigid-body states: link depth in the whole tree (world FK level by level)
    wdepth = [0] * L
    for l in range(L):
        wdepth[l] = 0 if lpar[l] < 0 else wdepth[lpar[l]] + 1
    glinks = [[l for l in range(L) if lgrp[l] == g] for g in range(G)]
    maxgl = max(len(x) for x in glinks)
    tlc = translating_locks(m, a)
    # link coms in their group's frame (3 per link, padded to 16 bytes): the
    # rigid-body force reduction's moment arms without link kinematics.  Not
    # for models whose epilogue moves locks in place (the links would move too)
    # link coms for the rigid-body force reduction; the Gogoro epilogue's
    # in-place seat moves do not maintain them (and its task applies no
    # per-link forces), the paper's do (rb_force_env shifts them)
    lcom = 0 if tlc["NTL"] and not fused_tasks(m) & 4 else (3 * L + 3) & ~3
    lines = [
        f"// AUTO-GENERATED by thormang_isaacgym_amd/model/codegen.py from model '{m.name}'. Do not edit.",
        "#pragma once",
        f"struct {cname} {{",
        f"  static constexpr unsigned long long hash = 0x{d.hash:016x}ULL;",
        f"  static constexpr int NG = {G}, NL = {L}, ND = {D}, NS = {S > 0 and S or 0}, NSA = {max(S, 1)};",
        f"  static constexpr int KC = {24 * G + 12 * S + tlc['KX'] + lcom};  // per-env composite floats (env-major, csrc CompLayout)",
        f"  static constexpr int KX = {tlc['KX']};  // of which the translating-lock extension (codegen translating_locks)",
        f"  static constexpr int LCOM = {1 if lcom else 0};  // link coms in their group frames (rigid-body force reduction)",
        f"  static constexpr int NTL = {tlc['NTL']}, tl_group = {tlc['tl_group']}, NAG = {len(tlc['ag'])}, "
        f"NASH = {len(tlc['ashape'])};",
        f"  static constexpr int tl_link[{max(tlc['NTL'], 1)}] = {_arr(tlc['tl_link'])};",
        f"  static constexpr int tl_dof[{max(tlc['NTL'], 1)}] = {_arr(tlc['tl_dof'])};",
        f"  static constexpr int link_tl[{L}] = {_arr(tlc['link_tl'])};",
        f"  static constexpr int ag_group[{max(len(tlc['ag']), 1)}] = {_arr([x[0] for x in tlc['ag']] or [0])};",
        f"  static constexpr int ag_mask[{max(len(tlc['ag']), 1)}] = {_arr([x[1] for x in tlc['ag']] or [0])};",
        f"  static constexpr int ash_shape[{max(len(tlc['ashape']), 1)}] = {_arr([x[0] for x in tlc['ashape']] or [0])};",
        f"  static constexpr int ash_mask[{max(len(tlc['ashape']), 1)}] = {_arr([x[1] for x in tlc['ashape']] or [0])};",
        f"  static constexpr int NROWS = {sum(n + (2 if n == 1 else 3) for n in nrows_n)};  // contact rows (normals + 3 friction per shape, 2 for one-point shapes)",
        f"  static constexpr int parent[{G}] = {_arr(a['group_parent'])};",
        f"  static constexpr int gdof[{G}] = {_arr(gdof)};",
        f"  static constexpr int jtype[{G}] = {_arr(gtype)};",
        f"  static constexpr float axis[{G}][3] = {_arr([_arr(x, _f) for x in gaxis])};",
        f"  static constexpr float gq[{G}][9] = {_arr([_arr(q.reshape(-1), _f) for q in gq])};  // joint-aligned frames",
        f"  static constexpr int shape_group[{max(S, 1)}] = {_arr(sgroup or [0])};",
        f"  static constexpr int shape_kind[{max(S, 1)}] = {_arr(list(a['shape_kind']) or [0])};",
        f"  static constexpr int shape_nrows[{max(S, 1)}] = {_arr(nrows_n or [0])};",
        f"  static constexpr float shape_params[{max(S, 1)}][4] = "
        f"{_arr([_arr(x, _f) for x in (a['shape_params'] if S else np.zeros((1, 4)))])};",
        f"  static constexpr float root_com[3] = {_arr(a['link_inertia'][0, 1:4], _f)};",
        # link tables for the compose step
        f"  static constexpr int link_parent[{L}] = {_arr(a['link_parent'])};",
        f"  static constexpr int link_group[{L}] = {_arr(a['link_group'])};",
        f"  static constexpr int link_dof[{L}] = {_arr(a['link_dof'])};",
        f"  static constexpr int link_jtype[{L}] = {_arr(a['link_jtype'])};",
        f"  static constexpr int link_is_group_root[{L}] = "
        f"{_arr([1 if i in set(int(x) for x in gr) else 0 for i in range(L)])};",
        f"  static constexpr float link_origin[{L}][12] = {_arr([_arr(x, _f) for x in a['link_origin']])};",
        f"  static constexpr float link_axis[{L}][3] = {_arr([_arr(x, _f) for x in a['link_axis']])};",
        f"  static constexpr float link_inertia[{L}][10] = {_arr([_arr(x, _f) for x in a['link_inertia']])};",
        f"  static constexpr int shape_link[{max(S, 1)}] = {_arr(list(a['shape_link']) or [0])};",
        f"  static constexpr float shape_pose[{max(S, 1)}][12] = "
        f"{_arr([_arr(x, _f) for x in (a['shape_pose'] if S else np.zeros((1, 12)))])};",
        f"  static constexpr int group_root[{G}] = {_arr(gr)};",
        f"  static constexpr unsigned char anc[{G}][{G}] = {_arr([_arr(r) for r in anc])};",
        f"  static constexpr int NCG = {max(len(cgroups), 1)}, MAXD = {maxd};",
        f"  static constexpr int cgroup[{max(len(cgroups), 1)}] = {_arr(cgroups or [0])};",
        f"  static constexpr int cpath_len[{max(len(cgroups), 1)}] = {_arr([depth[c] for c in cgroups] or [0])};",
        f"  static constexpr int cpath[{max(len(cgroups), 1)}][{maxd}] = "
        f"{_arr([_arr(p) for p in cpaths] or [_arr([0] * maxd)])};",
        f"  static constexpr int shape_cg[{max(S, 1)}] = {_arr(shape_cg or [0])};",
        f"  static constexpr int SL = {SL}, PAIR = {PAIR}, LPE = {LPE}, EPB = {EPB}, NSTEP = {len(sched)}, MAXC = {maxc};",
        f"  static constexpr int FUSED = {fused_tasks(m)};  // fused task epilogues: 1 walk, 2 Gogoro; 4 paper in-place seat",
        f"  static constexpr int sched[{len(sched)}][{SL}] = {_arr([_arr(r) for r in sched])};",
        f"  static constexpr int nchild[{G}] = {_arr([len(c) for c in children])};",
        f"  static constexpr int child[{G}][{maxc}] = {_arr([_arr(c + [-1] * (maxc - len(c))) for c in children])};",
        f"  static constexpr int dof_locked[{D}] = {_arr(a['dof_locked'])};",
        f"  static constexpr int NLEV = {max(level)}, MAXGL = {maxgl};",
        f"  static constexpr int link_level[{L}] = {_arr(level)};",
        f"  static constexpr int NDEPTH = {max(wdepth)};",
        f"  static constexpr int link_depth[{L}] = {_arr(wdepth)};",
        f"  static constexpr int group_nlinks[{G}] = {_arr([len(x) for x in glinks])};",
        f"  static constexpr int group_links[{G}][{maxgl}] = "
        f"{_arr([_arr(x + [-1] * (maxgl - len(x))) for x in glinks])};",
        "};",
        "",
    ]
    return "\n".join(lines)


def model_registry():
    """(c-name, Model) for every specialisation the library is built with."""
    out = []
    cdir = os.path.join(HERE, "compiled")
    for fn in sorted(os.listdir(cdir)):
        if fn.endswith(".json"):
            with open(os.path.join(cdir, fn)) as f:
                m = Model.from_json(f.read())
            out.append((f"Model_{m.name}", m))
    return out


def generate(out_dir: str) -> list:
    os.makedirs(out_dir, exist_ok=True)
    names = []
    for cname, m in model_registry():
        path = os.path.join(out_dir, f"{cname}.inc")
        text = emit(m, cname)
        if not os.path.exists(path) or open(path).read() != text:
            with open(path, "w") as f:
                f.write(text)
        names.append(cname)
    with open(os.path.join(out_dir, "models.inc"), "w") as f:
        f.write("// AUTO-GENERATED list of compiled model specialisations\n#pragma once\n")
        for n in names:
            f.write(f'#include "{n}.inc"\n')
        f.write("#define TG_FOR_EACH_MODEL(X) " + " ".join(f"X({n})" for n in names) + "\n")
    return names


if __name__ == "__main__":
    print(generate(os.path.join(os.path.dirname(HERE), "csrc", "generated")))

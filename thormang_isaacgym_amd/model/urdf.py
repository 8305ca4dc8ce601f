"""URDF -> articulation model compiler (host side, runs once per asset).

This replaces the asset half of IsaacGym's ``gym.load_asset`` as the reference
task uses it (``tasks/gogoro_new.py:196-231``): URDF parse, DOF enumeration and
the ``dof_name_to_id`` / rigid-body maps.  The output is a plain ``Model``
(JSON-serialisable) that the C-ABI consumes as flat arrays and that
``codegen.py`` folds into the specialised HIP step kernel.

Conventions (IsaacGym Preview-4 behaviour that cannot be checked offline,
SURVEY.md §7 hard part 7, recorded here once):

* bodies are the URDF links in depth-first order from the root link, children
  visited in joint-declaration order; DOFs are the non-fixed joints in the same
  order (this is the ``dof_state`` row order);
* a joint frame equals its child-link frame at q = 0 (URDF semantics); the axis
  is expressed in that frame;
* ``continuous`` joints are revolute without limits.

Beyond the raw tree the compiler builds **groups**: a group is a group-root link
plus every descendant reached through ``fixed`` or *locked* joints.  Locked
joints are the reference's limit-locked joints (``tasks/gogoro_new.py:257-262``
and the seat joints ``:562-572``): their per-env position changes only at reset,
so the dynamics run over groups (6 for the Gogoro rider model, 34 for the
stand-alone Thormang) and the per-env composite inertias are rebuilt by the
``compose`` kernel at reset.
"""
from __future__ import annotations

import json
import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field, asdict
from typing import Dict, List, Optional

import numpy as np

JOINT_FIXED, JOINT_REVOLUTE, JOINT_PRISMATIC = 0, 1, 2


def rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """URDF fixed-axis roll-pitch-yaw: R = Rz(y) Ry(p) Rx(r)."""
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([
        [cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
        [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
        [-sp, cp * sr, cp * cr],
    ])


def _vec(s: Optional[str], n=3, default=0.0):
    if s is None:
        return [default] * n
    v = [float(x) for x in s.split()]
    assert len(v) == n, s
    return v


@dataclass
class Shape:
    kind: str                 # "torus" | "box" | "sphere"
    link: str
    pos: List[float]          # in link frame
    rot: List[List[float]]    # 3x3, link <- shape
    params: List[float]       # torus: [R_major, r_minor] (axis = shape z); box: [hx,hy,hz]; sphere: [r]
    friction: float = 1.0


@dataclass
class Link:
    name: str
    mass: float
    com: List[float]
    inertia: List[float]      # ixx, iyy, izz, ixy, ixz, iyz about COM, link axes
    parent: int = -1          # parent link index (-1 root)
    joint: int = -1           # incoming joint index


@dataclass
class Joint:
    name: str
    jtype: int
    parent: int
    child: int
    origin_pos: List[float]
    origin_rot: List[List[float]]
    axis: List[float]
    lower: float = -math.inf
    upper: float = math.inf
    effort: float = 0.0
    velocity: float = 0.0
    has_limits: bool = False
    dof: int = -1             # index in dof order (-1 for fixed)


@dataclass
class Model:
    name: str
    links: List[Link] = field(default_factory=list)
    joints: List[Joint] = field(default_factory=list)
    shapes: List[Shape] = field(default_factory=list)
    dof_names: List[str] = field(default_factory=list)
    dof_joint: List[int] = field(default_factory=list)
    # grouping (filled by build_groups)
    locked: List[str] = field(default_factory=list)
    link_group: List[int] = field(default_factory=list)
    group_root: List[int] = field(default_factory=list)      # link index of each group root
    group_parent: List[int] = field(default_factory=list)    # parent group (-1 root)
    group_dof: List[int] = field(default_factory=list)       # active dof index of the group's joint (-1 root)
    active_dofs: List[int] = field(default_factory=list)     # dof indices, group order
    locked_dofs: List[int] = field(default_factory=list)

    # ----------------------------------------------------------------- helpers
    @property
    def num_dof(self) -> int:
        return len(self.dof_names)

    @property
    def num_bodies(self) -> int:
        return len(self.links)

    @property
    def num_groups(self) -> int:
        return len(self.group_root)

    def dof_name_to_id(self) -> Dict[str, int]:
        return {n: i for i, n in enumerate(self.dof_names)}

    def link_index(self, name: str) -> int:
        for i, l in enumerate(self.links):
            if l.name == name:
                return i
        raise KeyError(name)

    def forward_kinematics(self, q: Dict[str, float]) -> List[tuple]:
        """World (R, p) of every link with the root at the origin and joint
        positions ``q`` by dof name (missing names = 0)."""
        out = []
        for link in self.links:
            if link.parent < 0:
                out.append((np.eye(3), np.zeros(3)))
                continue
            j = self.joints[link.joint]
            R = np.asarray(j.origin_rot, np.float64)
            t = np.asarray(j.origin_pos, np.float64)
            th = float(q.get(j.name, 0.0)) if j.jtype != JOINT_FIXED else 0.0
            a = np.asarray(j.axis, np.float64)
            if j.jtype == JOINT_REVOLUTE:
                K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
                R = R @ (np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K)
            elif j.jtype == JOINT_PRISMATIC:
                t = t + R @ a * th
            Rp, pp = out[link.parent]
            out.append((Rp @ R, pp + Rp @ t))
        return out

    def lowest_point(self, q: Dict[str, float]) -> float:
        """Lowest z over all collision shapes (box corners / sphere / torus bottoms) at pose q."""
        fk = self.forward_kinematics(q)
        zmin = math.inf
        for s in self.shapes:
            R, p = fk[self.link_index(s.link)]
            Rs = R @ np.asarray(s.rot)
            c = p + R @ np.asarray(s.pos)
            if s.kind == "box":
                for sx in (-1, 1):
                    for sy in (-1, 1):
                        for sz in (-1, 1):
                            zmin = min(zmin, (c + Rs @ (np.array([sx, sy, sz]) * np.asarray(s.params)))[2])
            elif s.kind == "sphere":
                zmin = min(zmin, c[2] - s.params[0])
            else:
                zmin = min(zmin, c[2] - s.params[0] * np.sqrt(max(0.0, 1 - Rs[2, 2] ** 2)) - s.params[1])
        return zmin

    def to_json(self) -> str:
        return json.dumps(asdict(self), indent=1)

    @staticmethod
    def from_json(s: str) -> "Model":
        d = json.loads(s)
        m = Model(name=d["name"])
        m.links = [Link(**x) for x in d["links"]]
        m.joints = [Joint(**x) for x in d["joints"]]
        m.shapes = [Shape(**x) for x in d["shapes"]]
        for k in ("dof_names", "dof_joint", "locked", "link_group", "group_root", "group_parent",
                  "group_dof", "active_dofs", "locked_dofs"):
            setattr(m, k, d[k])
        return m

    # ---------------------------------------------------------------- grouping
    def build_groups(self, locked: List[str]) -> None:
        """Partition links into rigid groups joined by active joints.

        A link starts a new group when its incoming joint is an active
        (non-fixed, non-locked) DOF, or when it is the root."""
        names = set(locked)
        unknown = names - set(self.dof_names)
        if unknown:
            raise KeyError(f"locked joints not in model: {sorted(unknown)}")
        self.locked = [n for n in self.dof_names if n in names]
        self.link_group = [-1] * self.num_bodies
        self.group_root, self.group_parent, self.group_dof = [], [], []
        for li, link in enumerate(self.links):     # DFS order: parents first
            if link.parent < 0:
                starts = True
            else:
                j = self.joints[link.joint]
                starts = j.jtype != JOINT_FIXED and j.name not in names
            if starts:
                g = len(self.group_root)
                self.group_root.append(li)
                if link.parent < 0:
                    self.group_parent.append(-1)
                    self.group_dof.append(-1)
                else:
                    self.group_parent.append(self.link_group[link.parent])
                    self.group_dof.append(self.joints[link.joint].dof)
                self.link_group[li] = g
            else:
                self.link_group[li] = self.link_group[link.parent]
        self.active_dofs = [d for d in self.group_dof if d >= 0]
        self.locked_dofs = [self.dof_names.index(n) for n in self.locked]


def _parse_inertial(el) -> tuple:
    if el is None:
        return 0.0, [0.0, 0.0, 0.0], [0.0] * 6
    m = float(el.find("mass").get("value"))
    o = el.find("origin")
    com = _vec(o.get("xyz") if o is not None else None)
    rpy = _vec(o.get("rpy") if o is not None else None)
    ia = el.find("inertia").attrib
    I = np.array([[float(ia.get("ixx", 0)), float(ia.get("ixy", 0)), float(ia.get("ixz", 0))],
                  [float(ia.get("ixy", 0)), float(ia.get("iyy", 0)), float(ia.get("iyz", 0))],
                  [float(ia.get("ixz", 0)), float(ia.get("iyz", 0)), float(ia.get("izz", 0))]])
    R = rpy_to_matrix(*rpy)
    I = R @ I @ R.T
    return m, com, [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]


def fit_tire_torus(obj_path: str, scale: float) -> tuple:
    """Fit a torus (major R, minor r) to a tyre mesh whose spin axis is the
    mesh axis of least extent.  Returns (R, r, axis_index).  The crown radius
    R + r and the shoulder radius at |z| = 0.8*half-width pin the two
    parameters (r(0)=200 mm, r(+-37 mm)=190 mm)."""
    verts = []
    with open(obj_path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(x) for x in line.split()[1:4]])
    v = np.asarray(verts) * scale
    v -= (v.max(0) + v.min(0)) / 2
    ext = v.max(0) - v.min(0)
    ax = int(np.argmin(ext))
    z = v[:, ax]
    rho = np.linalg.norm(np.delete(v, ax, axis=1), axis=1)
    crown = rho[np.abs(z) < 0.05 * ext[ax]].max()
    zs = 0.8 * ext[ax] / 2
    band = np.abs(np.abs(z) - zs) < 0.05 * ext[ax]
    shoulder = rho[band].max()
    # R + r = crown ; R + sqrt(r^2 - zs^2) = shoulder
    d = crown - shoulder
    r = (zs * zs + d * d) / (2 * d)
    return crown - r, r, ax


def load_urdf(path: str, name: str, mesh_root: Optional[str] = None,
              inertia_override: Optional[Dict[str, tuple]] = None,
              extra_shapes: Optional[List[Shape]] = None,
              shape_friction: Optional[Dict[str, float]] = None) -> Model:
    root = ET.parse(path).getroot()
    link_el = {l.get("name"): l for l in root.findall("link")}
    joint_el = root.findall("joint")
    children: Dict[str, List] = {n: [] for n in link_el}
    child_names = set()
    for j in joint_el:
        children[j.find("parent").get("link")].append(j)
        child_names.add(j.find("child").get("link"))
    roots = [n for n in link_el if n not in child_names]
    if len(roots) != 1:
        raise ValueError(f"URDF must have one root link, found {roots}")

    m = Model(name=name)

    def add_link(lname: str, parent: int, joint: int):
        el = link_el[lname]
        mass, com, inertia = _parse_inertial(el.find("inertial"))
        if inertia_override and lname in inertia_override:
            inertia = list(inertia_override[lname])
        m.links.append(Link(lname, mass, com, inertia, parent, joint))
        return len(m.links) - 1

    stack = [(roots[0], -1, -1)]
    # iterative DFS preserving declaration order
    order = []

    def dfs(lname, parent, joint):
        li = add_link(lname, parent, joint)
        order.append(li)
        for j in children[lname]:
            jt = j.get("type")
            o = j.find("origin")
            xyz = _vec(o.get("xyz") if o is not None else None)
            rpy = _vec(o.get("rpy") if o is not None else None)
            a = j.find("axis")
            axis = _vec(a.get("xyz") if a is not None else None) if a is not None else [1.0, 0.0, 0.0]
            nrm = math.sqrt(sum(x * x for x in axis)) or 1.0
            axis = [x / nrm for x in axis]
            lim = j.find("limit")
            jtype = {"fixed": JOINT_FIXED, "revolute": JOINT_REVOLUTE, "continuous": JOINT_REVOLUTE,
                     "prismatic": JOINT_PRISMATIC}.get(jt)
            if jtype is None:
                raise ValueError(f"unsupported joint type {jt}")
            J = Joint(j.get("name"), jtype, li, -1, xyz, rpy_to_matrix(*rpy).tolist(), axis)
            if lim is not None:
                J.effort = float(lim.get("effort", 0.0))
                J.velocity = float(lim.get("velocity", 0.0))
                if jt != "continuous" and jtype != JOINT_FIXED:
                    J.lower = float(lim.get("lower", 0.0))
                    J.upper = float(lim.get("upper", 0.0))
                    J.has_limits = True
            if jtype != JOINT_FIXED:
                J.dof = len(m.dof_names)
                m.dof_names.append(J.name)
                m.dof_joint.append(len(m.joints))
            m.joints.append(J)
            ji = len(m.joints) - 1
            ci = dfs(j.find("child").get("link"), li, ji)
            m.joints[ji].child = ci
        return li

    dfs(*stack[0])

    # collision shapes
    for li, link in enumerate(m.links):
        for c in link_el[link.name].findall("collision"):
            g = list(c.find("geometry"))[0]
            o = c.find("origin")
            pos = _vec(o.get("xyz") if o is not None else None)
            R = rpy_to_matrix(*_vec(o.get("rpy") if o is not None else None))
            fr = (shape_friction or {}).get(link.name, 1.0)
            if g.tag == "mesh" and mesh_root is not None:
                fname = g.get("filename").split("/")[-1]
                sc = _vec(g.get("scale"), 3, 1.0)[0]
                Rt, rt, ax = fit_tire_torus(f"{mesh_root}/{fname}", sc)
                # align torus axis with shape z
                Pa = np.eye(3)[:, [(ax + 1) % 3, (ax + 2) % 3, ax]]
                m.shapes.append(Shape("torus", link.name, pos, (R @ Pa).tolist(), [Rt, rt], fr))
            elif g.tag == "box":
                s = _vec(g.get("size"))
                m.shapes.append(Shape("box", link.name, pos, R.tolist(), [x / 2 for x in s], fr))
            elif g.tag == "sphere":
                m.shapes.append(Shape("sphere", link.name, pos, R.tolist(), [float(g.get("radius"))], fr))
    for s in extra_shapes or []:
        m.shapes.append(s)
    return m

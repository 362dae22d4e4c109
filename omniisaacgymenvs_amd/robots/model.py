"""MJCF-subset model compiler: robot description -> the link tree libmi_sim.so simulates.

Replaces the reference's USD loading from Nucleus (robots/articulations/humanoid.py:40-67,
ant.py:40-67, cartpole.py:39-66), which is unavailable offline. The robot files under
``robots/assets/`` are AUTHORED for this build from the public MuJoCo-lineage humanoid / ant
models the reference's USDs were imported from; masses, inertias and joint parameters are
therefore this build's, not PhysX's.

Supported subset: <body pos quat>, <joint type=hinge|slide|free axis pos range damping
armature>, <freejoint>, <geom type=sphere|capsule size fromto pos density>,
<inertial pos mass diaginertia>, <site> (force-sensor reference), <default> joint/geom
attributes, compiler angle=degree|radian.

Compilation rules:
  * bodies without joints are welded into their parent (mass, inertia, geoms, sites);
  * a body with k joints becomes a chain of k one-DOF links; the link frame origin is the
    joint anchor, the last link carries the body's inertia / geoms / sites;
  * links are numbered in breadth-first body order, chains contiguous, so the joint DOF
    order is the BFS order ArticulationView reports
    (docs/transfering_policies_from_isaac_gym.md:39-54) and parent[l] < l.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import math
import os
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

import numpy as np

from .. import native as N

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


def asset_path(name: str) -> str:
    return os.path.join(ASSET_DIR, name)


# --------------------------------------------------------------------------------------
# small math (float64 on the host; cast to float32 for the device)
# --------------------------------------------------------------------------------------
def quat_to_mat(q) -> np.ndarray:
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def _floats(s: Optional[str], n: Optional[int] = None) -> Optional[np.ndarray]:
    if s is None:
        return None
    v = np.array([float(t) for t in s.split()], dtype=np.float64)
    if n is not None and v.size != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _sphere_inertia(r: float, rho: float):
    m = rho * 4.0 / 3.0 * math.pi * r ** 3
    i = 0.4 * m * r * r
    return m, np.diag([i, i, i])


def _capsule_inertia(r: float, h: float, rho: float):
    """Capsule with half-length h/2 along local z (MuJoCo's formula)."""
    mc = rho * math.pi * r * r * h
    ms = rho * 4.0 / 3.0 * math.pi * r ** 3
    izz = mc * r * r / 2.0 + ms * 0.4 * r * r
    ixx = mc * (r * r / 4.0 + h * h / 12.0) + ms * (0.4 * r * r + h * h / 4.0 + 3.0 * h * r / 8.0)
    return mc + ms, np.diag([ixx, ixx, izz])


def _frame_z_to(d: np.ndarray) -> np.ndarray:
    """Rotation whose z axis is the unit vector d."""
    z = d / np.linalg.norm(d)
    a = np.array([1.0, 0.0, 0.0]) if abs(z[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    x = np.cross(a, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


@dataclasses.dataclass
class _Geom:
    kind: int
    p0: np.ndarray
    p1: np.ndarray
    radius: float
    mass: float
    com: np.ndarray
    inertia: np.ndarray  # 3x3 about com, body frame


@dataclasses.dataclass
class _Joint:
    name: str
    kind: int
    axis: np.ndarray
    pos: np.ndarray
    lower: float
    upper: float
    damping: float
    armature: float


@dataclasses.dataclass
class _Body:
    name: str
    pos: np.ndarray
    quat: np.ndarray
    parent: Optional["_Body"]
    joints: List[_Joint]
    geoms: List[_Geom]
    sites: Dict[str, np.ndarray]
    children: List["_Body"]
    free: bool = False
    mass: float = 0.0
    com: np.ndarray = dataclasses.field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = dataclasses.field(default_factory=lambda: np.zeros((3, 3)))
    explicit_inertial: bool = False


@dataclasses.dataclass
class CompiledModel:
    """Link tree in the layout of mi_model_desc (include/mi_sim.h)."""

    name: str
    root_free: int
    parent: np.ndarray
    jtype: np.ndarray
    axis: np.ndarray
    pos: np.ndarray
    quat: np.ndarray
    mass: np.ndarray
    com: np.ndarray
    inertia: np.ndarray
    lower: np.ndarray
    upper: np.ndarray
    damping: np.ndarray
    armature: np.ndarray
    geom_link: np.ndarray
    geom_type: np.ndarray
    geom_p0: np.ndarray
    geom_p1: np.ndarray
    geom_radius: np.ndarray
    sensor_link: np.ndarray
    sensor_pos: np.ndarray
    pairs: np.ndarray
    dof_names: List[str]
    link_names: List[str]
    body_of_link: List[str]
    dyn_kind: int = N.MI_DYN_ARTICULATION
    cartpole: Dict[str, float] = dataclasses.field(default_factory=dict)

    @property
    def num_links(self) -> int:
        return int(self.parent.size)

    @property
    def num_dof(self) -> int:
        return self.num_links - 1

    @property
    def num_sensors(self) -> int:
        return int(self.sensor_link.size)

    @property
    def num_geoms(self) -> int:
        return int(self.geom_link.size)

    def dof_limits(self) -> np.ndarray:
        """[D, 2] (lower, upper) — ArticulationView.get_dof_limits()[0]."""
        return np.stack([self.lower[1:], self.upper[1:]], axis=1).astype(np.float32)

    def get_dof_index(self, name: str) -> int:
        return self.dof_names.index(name)

    def total_mass(self) -> float:
        return float(self.mass.sum())

    def to_desc(self) -> "ModelDesc":
        return ModelDesc(self)


class ModelDesc:
    """Keeps the numpy arrays alive while a ctypes MiModelDesc points into them."""

    def __init__(self, m: CompiledModel):
        # private copies: the ctypes struct points into these for the handle's lifetime
        f = lambda a: np.array(a, dtype=np.float32, order="C", copy=True)
        i = lambda a: np.array(a, dtype=np.int32, order="C", copy=True)
        self._keep = dict(
            parent=i(m.parent), jtype=i(m.jtype), axis=f(m.axis), pos=f(m.pos), quat=f(m.quat),
            mass=f(m.mass), com=f(m.com), inertia=f(m.inertia), lower=f(m.lower),
            upper=f(m.upper), damping=f(m.damping), armature=f(m.armature),
            geom_link=i(m.geom_link), geom_type=i(m.geom_type), geom_p0=f(m.geom_p0),
            geom_p1=f(m.geom_p1), geom_radius=f(m.geom_radius), sensor_link=i(m.sensor_link),
            sensor_pos=f(m.sensor_pos), pairs=i(m.pairs),
        )
        k = self._keep
        d = N.MiModelDesc()
        d.dyn_kind = m.dyn_kind
        d.root_free = m.root_free
        d.num_links = m.num_links
        d.num_geoms = m.num_geoms
        d.num_sensors = m.num_sensors
        d.num_pairs = int(m.pairs.shape[0])
        for name in ("axis", "pos", "quat", "mass", "com", "inertia", "lower", "upper", "damping",
                     "armature", "geom_p0", "geom_p1", "geom_radius", "sensor_pos"):
            setattr(d, name, N.fptr(k[name]))
        for name in ("parent", "jtype", "geom_link", "geom_type", "sensor_link", "pairs"):
            setattr(d, name, N.iptr(k[name]))
        cp = m.cartpole
        d.cart_mass = cp.get("cart_mass", 0.0)
        d.pole_mass = cp.get("pole_mass", 0.0)
        d.pole_com = cp.get("pole_com", 0.0)
        d.pole_inertia = cp.get("pole_inertia", 0.0)
        d.cart_damping = cp.get("cart_damping", 0.0)
        d.pole_damping = cp.get("pole_damping", 0.0)
        self.desc = d

    def ref(self):
        return C.byref(self.desc)


# --------------------------------------------------------------------------------------
# parsing
# --------------------------------------------------------------------------------------
class _Parser:
    def __init__(self, path: str):
        self.path = path
        root = ET.parse(path).getroot()
        self.model_name = root.get("model", os.path.basename(path))
        comp = root.find("compiler")
        self.degree = comp is None or comp.get("angle", "degree") == "degree"
        self.jdef = dict(damping="0", armature="0", limited="true")
        self.gdef = dict(density="1000")
        dflt = root.find("default")
        if dflt is not None:
            j = dflt.find("joint")
            g = dflt.find("geom")
            if j is not None:
                self.jdef.update(j.attrib)
            if g is not None:
                self.gdef.update(g.attrib)
        world = root.find("worldbody")
        bodies = world.findall("body")
        if len(bodies) != 1:
            raise ValueError("exactly one root body expected")
        self.root = self._body(bodies[0], None)

    def _angle(self, v: float) -> float:
        return math.radians(v) if self.degree else v

    def _body(self, el, parent) -> _Body:
        pos = _floats(el.get("pos", "0 0 0"), 3)
        quat = _floats(el.get("quat", "1 0 0 0"), 4)
        quat = quat / np.linalg.norm(quat)
        b = _Body(el.get("name", "body"), pos, quat, parent, [], [], {}, [])
        for ch in el:
            if ch.tag == "freejoint" or (ch.tag == "joint" and ch.get("type") == "free"):
                b.free = True
            elif ch.tag == "joint":
                a = dict(self.jdef)
                a.update(ch.attrib)
                kind = N.MI_JOINT_SLIDE if a.get("type", "hinge") == "slide" else N.MI_JOINT_HINGE
                axis = _floats(a.get("axis", "0 0 1"), 3)
                axis = axis / np.linalg.norm(axis)
                lo, hi = 1.0, 0.0
                if a.get("limited", "true") == "true" and "range" in a:
                    r = _floats(a["range"], 2)
                    if kind == N.MI_JOINT_HINGE:
                        r = np.array([self._angle(r[0]), self._angle(r[1])])
                    lo, hi = float(r[0]), float(r[1])
                b.joints.append(_Joint(a.get("name", f"{b.name}_j{len(b.joints)}"), kind, axis,
                                       _floats(a.get("pos", "0 0 0"), 3), lo, hi,
                                       float(a.get("damping", 0)), float(a.get("armature", 0))))
            elif ch.tag == "geom":
                b.geoms.append(self._geom(ch))
            elif ch.tag == "site":
                b.sites[ch.get("name", f"site{len(b.sites)}")] = _floats(ch.get("pos", "0 0 0"), 3)
            elif ch.tag == "inertial":
                b.explicit_inertial = True
                b.mass = float(ch.get("mass"))
                b.com = _floats(ch.get("pos", "0 0 0"), 3)
                b.inertia = np.diag(_floats(ch.get("diaginertia"), 3))
            elif ch.tag == "body":
                b.children.append(self._body(ch, b))
        if not b.explicit_inertial:
            self._mass_from_geoms(b)
        return b

    def _geom(self, el) -> _Geom:
        a = dict(self.gdef)
        a.update(el.attrib)
        kind = a.get("type", "sphere")
        size = _floats(a.get("size"))
        rho = float(a.get("density", 1000))
        if kind == "sphere":
            c = _floats(a.get("pos", "0 0 0"), 3)
            m, I = _sphere_inertia(size[0], rho)
            return _Geom(N.MI_GEOM_SPHERE, c, c.copy(), float(size[0]), m, c, I)
        if kind != "capsule":
            raise ValueError(f"unsupported geom type {kind!r}")
        if "fromto" in a:
            ft = _floats(a["fromto"], 6)
            p0, p1 = ft[:3], ft[3:]
        else:
            c = _floats(a.get("pos", "0 0 0"), 3)
            half = size[1]
            p0, p1 = c - np.array([0, 0, half]), c + np.array([0, 0, half])
        r = float(size[0])
        d = p1 - p0
        h = float(np.linalg.norm(d))
        m, Iloc = _capsule_inertia(r, h, rho)
        Rg = _frame_z_to(d) if h > 0 else np.eye(3)
        return _Geom(N.MI_GEOM_CAPSULE, p0, p1, r, m, 0.5 * (p0 + p1), Rg @ Iloc @ Rg.T)

    @staticmethod
    def _mass_from_geoms(b: _Body) -> None:
        m = sum(g.mass for g in b.geoms)
        if m <= 0:
            return
        com = sum(g.mass * g.com for g in b.geoms) / m
        I = np.zeros((3, 3))
        for g in b.geoms:
            d = g.com - com
            I += g.inertia + g.mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        b.mass, b.com, b.inertia = m, com, I


def _weld(child: _Body, parent: _Body) -> None:
    """Merge a joint-less child into its parent (frames: child -> parent body frame)."""
    R = quat_to_mat(child.quat)
    t = child.pos
    xf = lambda p: R @ p + t
    for g in child.geoms:
        parent.geoms.append(_Geom(g.kind, xf(g.p0), xf(g.p1), g.radius, g.mass, xf(g.com),
                                  R @ g.inertia @ R.T))
    for k, v in child.sites.items():
        parent.sites[k] = xf(v)
    mc, mp = child.mass, parent.mass
    if mc > 0:
        cc = xf(child.com)
        Ic = R @ child.inertia @ R.T
        m = mp + mc
        com = (mp * parent.com + mc * cc) / m
        I = np.zeros((3, 3))
        for (mm, c, Ii) in ((mp, parent.com, parent.inertia), (mc, cc, Ic)):
            d = c - com
            I += Ii + mm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        parent.mass, parent.com, parent.inertia = m, com, I
    for gc in child.children:
        # re-parent grandchildren: compose frames
        gc.pos = xf(gc.pos)
        gc.quat = _quat_mul(child.quat, gc.quat)
        gc.parent = parent
        parent.children.append(gc)


def _quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _weld_all(b: _Body) -> None:
    changed = True
    while changed:
        changed = False
        for ch in list(b.children):
            if not ch.joints and not ch.free:
                b.children.remove(ch)
                _weld(ch, b)
                changed = True
    for ch in b.children:
        _weld_all(ch)


def segment_distance(a0, a1, b0, b1):
    """Closest distance between segments [a0, a1] and [b0, b1] (points allowed), numpy."""
    d1, d2, r = a1 - a0, b1 - b0, a0 - b0
    a, e, f = d1 @ d1, d2 @ d2, d2 @ r
    if a <= 1e-12 and e <= 1e-12:
        return float(np.linalg.norm(r))
    if a <= 1e-12:
        s, t = 0.0, np.clip(f / e, 0.0, 1.0)
    else:
        c = d1 @ r
        if e <= 1e-12:
            s, t = np.clip(-c / a, 0.0, 1.0), 0.0
        else:
            b = d1 @ d2
            den = a * e - b * b
            s = np.clip((b * f - c * e) / den, 0.0, 1.0) if den > 1e-12 else 0.0
            t = (b * s + f) / e
            if t < 0.0:
                s, t = np.clip(-c / a, 0.0, 1.0), 0.0
            elif t > 1.0:
                s, t = np.clip((b - c) / a, 0.0, 1.0), 1.0
    return float(np.linalg.norm((a0 + d1 * s) - (b0 + d2 * t)))


def _self_collision_pairs(order, min_gap: float) -> List[tuple]:
    """Geom pairs that may self-collide, in compiled geom order: geoms of different bodies that
    are not joint-connected (PhysX does not collide a link with its parent), minus pairs whose
    surfaces are closer than ``min_gap`` in the default pose (initial-overlap filter)."""
    Rw, pw = {}, {}
    for b in order:
        if b.parent is None:
            Rw[b.name], pw[b.name] = np.eye(3), np.zeros(3)
        else:
            Rp, pp = Rw[b.parent.name], pw[b.parent.name]
            Rw[b.name] = Rp @ quat_to_mat(b.quat)
            pw[b.name] = pp + Rp @ b.pos
    geoms = []   # (body, world p0, world p1, radius) in compiled geom order
    for b in order:
        for g in b.geoms:
            geoms.append((b, pw[b.name] + Rw[b.name] @ g.p0, pw[b.name] + Rw[b.name] @ g.p1, g.radius))
    pairs = []
    for i in range(len(geoms)):
        for j in range(i + 1, len(geoms)):
            bi, bj = geoms[i][0], geoms[j][0]
            if bi is bj or bi.parent is bj or bj.parent is bi:
                continue
            gap = segment_distance(geoms[i][1], geoms[i][2], geoms[j][1], geoms[j][2]) - \
                geoms[i][3] - geoms[j][3]
            if gap >= min_gap:
                pairs.append((i, j))
    return pairs


def compile_mjcf(path: str, sensor_bodies: Optional[List[str]] = None,
                 self_collision_pairs: Optional[List[tuple]] = None,
                 self_collision: bool = False, self_collision_min_gap: float = 0.05) -> CompiledModel:
    """Compile an MJCF-subset file. ``sensor_bodies`` lists force-sensor bodies in output
    order (the wrench reference is the body's first site, else its frame origin).
    ``self_collision``: generate the self-collision geom pairs (see _self_collision_pairs)."""
    p = _Parser(path)
    root = p.root
    _weld_all(root)
    # breadth-first body order
    order: List[_Body] = []
    queue = [root]
    while queue:
        b = queue.pop(0)
        order.append(b)
        queue.extend(b.children)
    parent, jtype, axis, pos, quat = [-1], [0], [[0, 0, 1]], [[0, 0, 0]], [[1, 0, 0, 0]]
    mass, com, inertia = [root.mass], [root.com], [root.inertia]
    lower, upper, damping, armature = [1.0], [0.0], [0.0], [0.0]
    dof_names, link_names, body_of_link = [], ["root"], [root.name]
    last_link = {root.name: 0}
    last_anchor = {root.name: np.zeros(3)}
    for b in order[1:]:
        if not b.joints:
            raise ValueError(f"body {b.name} has no joint after welding")
        Pb = b.parent
        pl = last_link[Pb.name]
        pa = last_anchor[Pb.name]
        Rb = quat_to_mat(b.quat)
        prev_anchor = None
        for k, j in enumerate(b.joints):
            if k == 0:
                pos.append(b.pos - pa + Rb @ j.pos)
                quat.append(b.quat)
                parent.append(pl)
            else:
                pos.append(j.pos - prev_anchor)
                quat.append(np.array([1.0, 0, 0, 0]))
                parent.append(len(parent) - 1)
            prev_anchor = j.pos
            jtype.append(j.kind)
            axis.append(j.axis)
            lower.append(j.lower)
            upper.append(j.upper)
            damping.append(j.damping)
            armature.append(j.armature)
            dof_names.append(j.name)
            link_names.append(j.name)
            body_of_link.append(b.name)
            last = k == len(b.joints) - 1
            mass.append(b.mass if last else 0.0)
            com.append(b.com - j.pos if last else np.zeros(3))
            inertia.append(b.inertia if last else np.zeros((3, 3)))
        last_link[b.name] = len(parent) - 1
        last_anchor[b.name] = b.joints[-1].pos
    body_by_name = {b.name: b for b in order}
    gl, gt, g0, g1, gr = [], [], [], [], []
    for b in order:
        li, a = last_link[b.name], last_anchor[b.name]
        for g in b.geoms:
            gl.append(li)
            gt.append(g.kind)
            g0.append(g.p0 - a)
            g1.append(g.p1 - a)
            gr.append(g.radius)
    sl, sp = [], []
    for name in sensor_bodies or []:
        b = body_by_name[name]
        site = next(iter(b.sites.values())) if b.sites else np.zeros(3)
        sl.append(last_link[name])
        sp.append(site - last_anchor[name])
    if self_collision and self_collision_pairs is None:
        self_collision_pairs = _self_collision_pairs(order, self_collision_min_gap)
    pairs = np.array(self_collision_pairs or [], dtype=np.int32).reshape(-1, 2)

    def sym6(I):
        return [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]

    f = lambda v, shape: np.asarray(v, dtype=np.float64).reshape(shape)
    L = len(parent)
    return CompiledModel(
        name=p.model_name, root_free=1 if root.free else 0,
        parent=np.array(parent, dtype=np.int32), jtype=np.array(jtype, dtype=np.int32),
        axis=f(axis, (L, 3)), pos=f(pos, (L, 3)), quat=f(quat, (L, 4)), mass=f(mass, (L,)),
        com=f(com, (L, 3)), inertia=f([sym6(I) for I in inertia], (L, 6)),
        lower=f(lower, (L,)), upper=f(upper, (L,)), damping=f(damping, (L,)),
        armature=f(armature, (L,)),
        geom_link=np.array(gl, dtype=np.int32), geom_type=np.array(gt, dtype=np.int32),
        geom_p0=f(g0, (-1, 3)), geom_p1=f(g1, (-1, 3)), geom_radius=f(gr, (-1,)),
        sensor_link=np.array(sl, dtype=np.int32), sensor_pos=f(sp, (-1, 3)), pairs=pairs,
        dof_names=dof_names, link_names=link_names, body_of_link=body_of_link,
    )


def load_robot(name: str) -> CompiledModel:
    """The three robots of the hot path with their task-side sensor lists."""
    if name == "Humanoid":
        # Humanoid.yaml:80 enable_self_collisions: True -> generate the pair list (used only
        # when the sim params enable self-collisions)
        return compile_mjcf(asset_path("humanoid.xml"), sensor_bodies=["right_foot", "left_foot"],
                            self_collision=True)
    if name == "Ant":
        return compile_mjcf(asset_path("ant.xml"), sensor_bodies=[
            "front_left_foot", "front_right_foot", "left_back_foot", "right_back_foot"])
    if name == "Cartpole":
        m = compile_mjcf(asset_path("cartpole.xml"))
        m.dyn_kind = N.MI_DYN_CARTPOLE
        m.cartpole = dict(cart_mass=float(m.mass[1]), pole_mass=float(m.mass[2]),
                          pole_com=float(m.com[2][2]), pole_inertia=float(m.inertia[2][1]),
                          cart_damping=float(m.damping[1]), pole_damping=float(m.damping[2]))
        return m
    raise KeyError(name)

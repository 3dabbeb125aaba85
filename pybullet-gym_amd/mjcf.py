"""MJCF -> static articulated-robot tables (the "model compiler").

The reference hands an MJCF path to ``pybullet.loadMJCF`` (``robot_bases.py:108,116``)
and then walks the resulting multibody with ``getJointInfo`` in
``XmlBasedRobot.addToScene`` (``robot_bases.py:32-91``).  pybullet's MJCF importer is
third-party C++ that is not in /root/reference, so every rule it applies is restated
here as an explicit, documented choice (all
unpinned by anything in this container):

* B2 topology: a root body without joints becomes a floating base (Ant, Humanoid); a
  root body with joints hangs off a fixed, massless world base (Hopper, HalfCheetah,
  InvertedPendulum).  A body with k joints becomes k chained links, the first k-1 of
  them massless dummies named ``<body>_dummy<i>``; a body with no joint becomes a
  ``jointfix_*`` fixed link.  Links are numbered in MJCF depth-first order, which is
  the order ``addToScene`` enumerates them (``robot_bases.py:60``).
* B3 mass: geom volume x 1000 (capsule volume includes both hemispheres; the geom
  ``density`` attribute is not read: Ant's density="5" would leave a 0.9 kg ant on
  250 N m motors), ``<inertial mass=..>`` overrides the body mass, ``settotalmass`` is not
  read.  Inertia is Bullet's compound-shape approximation, not the solid's: the mass
  times the box inertia of the link's collision AABB in the link frame
  (btCompoundShape::calculateLocalInertia, applied by URDF2Bullet when loadMJCF is not
  given URDF_USE_INERTIA_FROM_FILE -- robot_bases.py:108,116 pass only self-collision
  flags), diagonal in the link axes.  Joint ``armature`` is not modelled (btMultiBody has
  none).  These four choices are backed by the reference's pretrained roboschool
  policies (tests/test_policies.py): each one raises or holds every policy's score on the
  oracle (Hopper 60 -> 1130 mean return, Ant -119 -> 734, InvertedDoublePendulum
  3125 -> 4368) against the exact-solid / armature / density / settotalmass rules.
* B4 collision: every robot geom whose contype or conaffinity is non-zero collides
  with the floor; robot-robot pairs follow MuJoCo's contype/conaffinity rule and
  exclude every ancestor pair (URDF_USE_SELF_COLLISION_EXCLUDE_ALL_PARENTS,
  ``robot_bases.py:116``).
* B5 friction: geom friction[0] times the floor's lateral friction 0.8
  (``scene_stadium.py:33``); restitution 0 x 0.5 = 0, except where the env sets the links'
  material itself (HalfCheetahMuJoCo: restitution 0.5 x 0.5, spinning and rolling friction
  0.1 x 0.8 -- codegen.py).
* B6 damping: the joint element's own ``damping`` attribute, applied as -d*qdot from each
  sub-step's velocity (pybullet applies it per stepSimulation; per sub-step is the stable
  choice at dt/4); a ``<default><joint damping=..>`` is not inherited (pybullet's importer takes
  only ``limited`` from joint defaults).  Evidence: with inherited damping 1 the
  pretrained swing-up policy never swings the pole up (mean return -666); without it,
  878 -- and InvertedDoublePendulum 4368 -> 6491 (tests/test_policies.py).
* B7 stiffness: the joint element's own ``stiffness`` attribute as a spring to q = 0,
  tau -= k*q from each sub-step's position (explicit, beside B6's damping); not inherited
  from ``<default>``.  Evidence (round 3): the pretrained HalfCheetah
  policy runs every 64-episode rollout to the 1,000-step limit with it (mean return 729 ->
  1,301; without it episodes end at 702 steps on average), Humanoid 30 -> 37; no other
  robot's MJCF sets a non-zero stiffness.
* The base frame is the base's centre of mass (pybullet reports base and link
  positions of the inertial frame); link frames are MJCF body frames and keep a COM
  offset.  Inertial frames are not rotated to principal axes.

The compiled tables are committed as ``models/<robot>.json`` and as the C++ header
``csrc/models_gen.h`` (see ``codegen.py``) so that nothing on the GPU box reads the
reference's asset tree.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

JOINT_REVOLUTE = 0   # pybullet.JOINT_REVOLUTE
JOINT_PRISMATIC = 1  # pybullet.JOINT_PRISMATIC
JOINT_FIXED = 4      # pybullet.JOINT_FIXED

GEOM_SPHERE = 0
GEOM_CAPSULE = 1
GEOM_BOX = 2       # URDF robots (urdf.py): half extents + rotation in the link frame
GEOM_CYLINDER = 3  # URDF robots: a Z cylinder, p0 / p1 its cap centres

FLOOR_FRICTION = 0.8  # scene_stadium.py:33
FLOOR_RESTITUTION = 0.5  # scene_stadium.py:33


# ----------------------------------------------------------------------------- math
def quat_wxyz_to_mat(q) -> np.ndarray:
    w, x, y, z = [float(v) for v in q]
    n = math.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / n, x / n, y / n, z / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def mat_to_quat_xyzw(m: np.ndarray) -> Tuple[float, float, float, float]:
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w = 0.25 * s
        x = (m[2, 1] - m[1, 2]) / s
        y = (m[0, 2] - m[2, 0]) / s
        z = (m[1, 0] - m[0, 1]) / s
    elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        s = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        w = (m[2, 1] - m[1, 2]) / s
        x = 0.25 * s
        y = (m[0, 1] + m[1, 0]) / s
        z = (m[0, 2] + m[2, 0]) / s
    elif m[1, 1] > m[2, 2]:
        s = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        w = (m[0, 2] - m[2, 0]) / s
        x = (m[0, 1] + m[1, 0]) / s
        y = 0.25 * s
        z = (m[1, 2] + m[2, 1]) / s
    else:
        s = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
        w = (m[1, 0] - m[0, 1]) / s
        x = (m[0, 2] + m[2, 0]) / s
        y = (m[1, 2] + m[2, 1]) / s
        z = 0.25 * s
    return (x, y, z, w)


def axisangle_to_mat(axis, angle) -> np.ndarray:
    a = np.asarray(axis, dtype=float)
    a = a / np.linalg.norm(a)
    s, c = math.sin(angle / 2), math.cos(angle / 2)
    return quat_wxyz_to_mat([c, a[0] * s, a[1] * s, a[2] * s])


# ----------------------------------------------------------------------------- data
@dataclass
class Geom:
    name: str
    kind: int                 # GEOM_SPHERE / GEOM_CAPSULE
    radius: float
    p0: np.ndarray            # segment endpoints in the owning link frame (sphere: p0 == p1)
    p1: np.ndarray
    friction: float
    contype: int
    conaffinity: int
    mass: float = 0.0
    half: Optional[np.ndarray] = None  # box / cylinder (urdf.py): half extents in the geom frame
    rot: Optional[np.ndarray] = None   # box / cylinder: geom frame in the link frame


@dataclass
class Link:
    name: str                 # pybullet link name (getJointInfo[12])
    joint_name: str           # getJointInfo[1]
    parent: int               # link index, -1 = base
    jtype: int
    offset_pos: np.ndarray    # link frame origin in parent link frame at q=0
    offset_rot: np.ndarray    # 3x3
    axis: np.ndarray          # joint axis, link frame
    anchor: np.ndarray        # joint anchor, link frame
    lower: float = 0.0
    upper: float = -1.0       # lower > upper -> no limits (pybullet convention)
    limited: bool = False
    damping: float = 0.0
    stiffness: float = 0.0    # B7: spring to q = 0 (N m / rad or N / m)
    armature: float = 0.0
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))
    geoms: List[Geom] = field(default_factory=list)
    body: str = ""
    dof: int = -1             # joint dof index (0..NJ-1) or -1 for fixed
    max_velocity: float = 0.0  # getJointInfo maxVelocity (URDF <limit velocity>; MJCF joints: 0)


@dataclass
class RobotModel:
    name: str
    floating: bool
    base_name: str
    base_mass: float
    base_inertia: np.ndarray
    base_pos: np.ndarray      # world position of the base (COM) frame at load
    base_rot: np.ndarray
    base_geoms: List[Geom]
    links: List[Link]

    @property
    def n_links(self) -> int:
        return len(self.links)

    @property
    def n_joint_dofs(self) -> int:
        return sum(1 for l in self.links if l.jtype != JOINT_FIXED)

    def link_index(self, name: str) -> int:
        for i, l in enumerate(self.links):
            if l.name == name:
                return i
        raise KeyError(name)

    def dof_link(self) -> List[int]:
        return [i for i, l in enumerate(self.links) if l.jtype != JOINT_FIXED]

    def total_mass(self) -> float:
        return self.base_mass + sum(l.mass for l in self.links)

    def ancestors(self, li: int) -> List[int]:
        out = []
        p = self.links[li].parent
        while p >= 0:
            out.append(p)
            p = self.links[p].parent
        return out


# ----------------------------------------------------------------------------- inertia
def geom_mass_props(kind: int, radius: float, p0: np.ndarray, p1: np.ndarray, density: float):
    """Mass, centre and inertia (about the centre, link frame) of a solid sphere/capsule."""
    r = radius
    c = 0.5 * (p0 + p1)
    if kind == GEOM_SPHERE:
        m = density * 4.0 / 3.0 * math.pi * r ** 3
        return m, c, np.eye(3) * (0.4 * m * r * r)
    seg = p1 - p0
    length = float(np.linalg.norm(seg))
    h = 0.5 * length
    mc = density * math.pi * r * r * length
    ms = density * 4.0 / 3.0 * math.pi * r ** 3
    i_axial = 0.5 * mc * r * r + 0.4 * ms * r * r
    i_perp = mc * (3 * r * r + length * length) / 12.0 + ms * (83.0 / 320.0 * r * r + (h + 3.0 * r / 8.0) ** 2)
    if length < 1e-12:
        u = np.array([0.0, 0.0, 1.0])
    else:
        u = seg / length
    inertia = i_perp * np.eye(3) + (i_axial - i_perp) * np.outer(u, u)
    return mc + ms, c, inertia


def combine_mass(parts):
    """parts: list of (m, c, I_about_c) -> (M, com, I_about_com)."""
    M = sum(p[0] for p in parts)
    if M <= 0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    com = sum(p[0] * p[1] for p in parts) / M
    inertia = np.zeros((3, 3))
    for m, c, ic in parts:
        d = c - com
        inertia += ic + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return M, com, inertia


PYBULLET_MJCF_DENSITY = 1000.0
APPLY_SETTOTALMASS = False


def _shortest_arc(u: np.ndarray) -> np.ndarray:
    """Rotation taking +z to unit vector u (Bullet's shortestArcQuat, as the MJCF importer
    orients a fromto capsule: a btCapsuleShapeZ in a child transform)."""
    z = np.array([0.0, 0.0, 1.0])
    v = np.cross(z, u)
    s = float(np.linalg.norm(v))
    c = float(np.dot(z, u))
    if s < 1e-12:
        return np.eye(3) if c > 0 else np.diag([1.0, -1.0, -1.0])
    k = v / s
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    ang = math.atan2(s, c)
    return np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * (K @ K)


def collision_aabb(geoms) -> Tuple[np.ndarray, np.ndarray]:
    """AABB (link frame) of a link's collision shapes as Bullet computes it: each capsule is
    a Z capsule with half extents (r, r, r + h/2) whose box is rotated into the link frame
    (btCapsuleShape::getAabb: |R| he), a sphere is +-r; the compound takes the union."""
    lo = np.full(3, np.inf)
    hi = np.full(3, -np.inf)
    for g in geoms:
        c = 0.5 * (g.p0 + g.p1)
        if g.kind == GEOM_SPHERE:
            ext = np.full(3, g.radius)
        else:
            seg = g.p1 - g.p0
            L = float(np.linalg.norm(seg))
            u = seg / L if L > 1e-12 else np.array([0.0, 0.0, 1.0])
            ext = np.abs(_shortest_arc(u)) @ np.array([g.radius, g.radius, g.radius + 0.5 * L])
        lo = np.minimum(lo, c - ext)
        hi = np.maximum(hi, c + ext)
    return lo, hi


def bullet_compound_inertia(geoms, mass: float) -> np.ndarray:
    """btCompoundShape::calculateLocalInertia: "approximation: take the inertia from the
    aabb" -- the solid box of the compound's AABB, I = m/12 (l_y^2 + l_z^2, ...), diagonal in
    the link axes (the inertial frame of an MJCF body without <inertial> is unrotated)."""
    lo, hi = collision_aabb(geoms)
    l = hi - lo
    return np.diag([mass / 12.0 * (l[1] ** 2 + l[2] ** 2), mass / 12.0 * (l[0] ** 2 + l[2] ** 2),
                    mass / 12.0 * (l[0] ** 2 + l[1] ** 2)])


# ----------------------------------------------------------------------------- parser
def _floats(s: Optional[str], n: Optional[int] = None) -> Optional[np.ndarray]:
    if s is None:
        return None
    v = np.array([float(x) for x in s.split()], dtype=float)
    if n is not None and len(v) < n:
        v = np.concatenate([v, np.zeros(n - len(v))])
    return v


# Rule-study switch (tools/physics_rules.py, round 5): joint damping inherited from <default>.  The
# product tables (codegen.py) are compiled with it off (B6).
INHERIT_DEFAULT_DAMPING = False


class _Ctx:
    def __init__(self, root: ET.Element):
        comp = root.find("compiler")
        self.degree = True
        self.global_coords = False
        self.settotalmass = None
        if comp is not None:
            self.degree = comp.get("angle", "degree") == "degree"
            self.global_coords = comp.get("coordinate", "local") == "global"
            if comp.get("settotalmass") is not None:
                self.settotalmass = float(comp.get("settotalmass"))
        self.djoint: Dict[str, str] = {}
        self.dgeom: Dict[str, str] = {}
        d = root.find("default")
        if d is not None:
            j = d.find("joint")
            g = d.find("geom")
            if j is not None:
                self.djoint = dict(j.attrib)
            if g is not None:
                self.dgeom = dict(g.attrib)

    def angle(self, v: float) -> float:
        return math.radians(v) if self.degree else v

    def jattr(self, el, key, default=None):
        return el.get(key, self.djoint.get(key, default))

    def gattr(self, el, key, default=None):
        return el.get(key, self.dgeom.get(key, default))


def _frame_of(ctx: _Ctx, el) -> Tuple[np.ndarray, np.ndarray]:
    pos = _floats(el.get("pos"), 3)
    pos = np.zeros(3) if pos is None else pos
    rot = np.eye(3)
    if el.get("quat") is not None:
        rot = quat_wxyz_to_mat(_floats(el.get("quat")))
    elif el.get("axisangle") is not None:
        aa = _floats(el.get("axisangle"))
        rot = axisangle_to_mat(aa[:3], ctx.angle(aa[3]))
    elif el.get("euler") is not None:
        raise NotImplementedError("euler frames are not used by the locomotion assets")
    return pos, rot


def _parse_geom(ctx: _Ctx, g) -> Tuple[Geom, float]:
    kind_s = ctx.gattr(g, "type", "sphere")
    size = _floats(ctx.gattr(g, "size"))
    density = PYBULLET_MJCF_DENSITY  # B3: the geom density attribute is not read
    fr = _floats(ctx.gattr(g, "friction", "1 0.005 0.0001"))
    contype = int(ctx.gattr(g, "contype", "1"))
    conaff = int(ctx.gattr(g, "conaffinity", "1"))
    name = g.get("name", "")
    if kind_s == "sphere":
        pos, _ = _frame_of(ctx, g)
        geom = Geom(name, GEOM_SPHERE, float(size[0]), pos.copy(), pos.copy(), float(fr[0]), contype, conaff)
    elif kind_s == "capsule":
        if g.get("fromto") is not None:
            ft = _floats(g.get("fromto"))
            p0, p1 = ft[:3].copy(), ft[3:6].copy()
        else:
            pos, rot = _frame_of(ctx, g)
            half = float(size[1])
            ax = rot @ np.array([0.0, 0.0, half])
            p0, p1 = pos - ax, pos + ax
        geom = Geom(name, GEOM_CAPSULE, float(size[0]), p0, p1, float(fr[0]), contype, conaff)
    else:
        raise NotImplementedError(f"geom type {kind_s}")
    return geom, density


def _transform_geom(g: Geom, pos: np.ndarray, rot: np.ndarray) -> Geom:
    """Express a geom given in frame F in the frame where F = (pos, rot)."""
    return Geom(g.name, g.kind, g.radius, pos + rot @ g.p0, pos + rot @ g.p1, g.friction, g.contype, g.conaffinity, g.mass)


def compile_mjcf(path: str, robot_name: str) -> RobotModel:
    """Compile one MJCF file (reference asset) into a RobotModel."""
    root = ET.parse(path).getroot()
    ctx = _Ctx(root)
    world = root.find("worldbody")
    roots = world.findall("body")
    assert len(roots) == 1, "locomotion assets have a single root body"
    rb = roots[0]

    links: List[Link] = []
    body_mass: Dict[str, Tuple[float, np.ndarray, np.ndarray, List[Geom]]] = {}

    def body_inertial(b) -> Tuple[float, np.ndarray, np.ndarray, List[Geom]]:
        geoms, parts = [], []
        for g in b.findall("geom"):
            geom, dens = _parse_geom(ctx, g)
            m, c, ic = geom_mass_props(geom.kind, geom.radius, geom.p0, geom.p1, dens)
            geom.mass = m
            geoms.append(geom)
            parts.append((m, c, ic))
        M, com, inertia = combine_mass(parts)
        inert = b.find("inertial")
        if inert is not None and inert.get("mass") is not None:
            m_new = float(inert.get("mass"))
            scale = m_new / M if M > 0 else 0.0
            M, inertia = m_new, inertia * scale
        if geoms:
            inertia = bullet_compound_inertia(geoms, M)
        return M, com, inertia, geoms

    def joint_info(j, rot_body_to_link=np.eye(3)):
        jt = j.get("type", "hinge")
        jtype = JOINT_REVOLUTE if jt == "hinge" else JOINT_PRISMATIC if jt == "slide" else None
        if jtype is None:
            raise NotImplementedError(jt)
        axis = _floats(j.get("axis"), 3)
        axis = np.array([0.0, 0.0, 1.0]) if axis is None else axis
        axis = axis / np.linalg.norm(axis)
        anchor = _floats(j.get("pos"), 3)
        anchor = np.zeros(3) if anchor is None else anchor
        limited = ctx.jattr(j, "limited", "false") == "true"
        lo, hi = 0.0, -1.0
        rng = j.get("range")
        if limited and rng is not None:
            r = _floats(rng)
            if jtype == JOINT_REVOLUTE:
                lo, hi = ctx.angle(r[0]), ctx.angle(r[1])
            else:
                lo, hi = float(r[0]), float(r[1])
            if not lo < hi:
                limited = False
        else:
            limited = False
        return dict(jtype=jtype, axis=axis, anchor=anchor, lower=lo if limited else 0.0,
                    upper=hi if limited else -1.0, limited=limited,
                    # B6: the joint's own attribute only (INHERIT_DEFAULT_DAMPING: the rule study's
                    # alternative, <default> inherited; tools/physics_rules.py, never the product tables)
                    damping=float((ctx.jattr(j, "damping", "0") if INHERIT_DEFAULT_DAMPING else j.get("damping", "0"))),
                    stiffness=float(j.get("stiffness", "0")),  # B7: likewise
                    armature=0.0,  # B3: btMultiBody has no armature
                    joint_name=j.get("name"))

    def add_body(b, parent_link: int, parent_pos_shift: np.ndarray):
        """Add the links of body b; returns nothing. parent_pos_shift = origin of parent link
        frame expressed in the parent's MJCF body frame (non-zero only for a COM-shifted base)."""
        bpos, brot = _frame_of(ctx, b)
        if ctx.global_coords:
            assert np.allclose(bpos, 0) and np.allclose(brot, np.eye(3)), "global coords need pos-less bodies"
        M, com, inertia, geoms = body_inertial(b)
        joints = b.findall("joint")
        name = b.get("name")
        first = len(links)
        if not joints:
            jn = f"jointfix_{len(links)}_{name}"
            links.append(Link(name=name, joint_name=jn, parent=parent_link, jtype=JOINT_FIXED,
                              offset_pos=bpos - parent_pos_shift, offset_rot=brot,
                              axis=np.zeros(3), anchor=np.zeros(3), body=name))
        else:
            for k, j in enumerate(joints):
                ji = joint_info(j)
                last = k == len(joints) - 1
                lname = name if last else f"{name}_dummy{k}"
                if k == 0:
                    op, orot, par = bpos - parent_pos_shift, brot, parent_link
                else:
                    op, orot, par = np.zeros(3), np.eye(3), len(links) - 1
                links.append(Link(name=lname, parent=par, offset_pos=op, offset_rot=orot, body=name, **ji))
        real = links[-1]
        real.mass, real.com, real.inertia, real.geoms = M, com, inertia, geoms
        # dummies of a multi-joint body sit at the body origin, massless
        for l in links[first:-1]:
            l.com = np.zeros(3)
        me = len(links) - 1
        for child in b.findall("body"):
            add_body(child, me, np.zeros(3))

    root_joints = rb.findall("joint")
    M, com, inertia, geoms = body_inertial(rb)
    rpos, rrot = _frame_of(ctx, rb)
    if not root_joints:
        # floating base at the root body's COM
        base = dict(floating=True, base_name=rb.get("name"), base_mass=M, base_inertia=inertia,
                    base_pos=rpos + rrot @ com, base_rot=rrot,
                    base_geoms=[_transform_geom(g, -com, np.eye(3)) for g in geoms])
        for child in rb.findall("body"):
            add_body(child, -1, com)
    else:
        base = dict(floating=False, base_name="world", base_mass=0.0, base_inertia=np.zeros((3, 3)),
                    base_pos=np.zeros(3), base_rot=np.eye(3), base_geoms=[])
        add_body(rb, -1, np.zeros(3))

    model = RobotModel(name=robot_name, links=links, **base)
    if ctx.settotalmass is not None and APPLY_SETTOTALMASS:
        s = ctx.settotalmass / model.total_mass()
        model.base_mass *= s
        model.base_inertia = model.base_inertia * s
        for l in model.links:
            l.mass *= s
            l.inertia = l.inertia * s
    d = 0
    for l in model.links:
        if l.jtype != JOINT_FIXED:
            l.dof = d
            d += 1
    return model


# ----------------------------------------------------------------------------- kinematics
def link_world_frames(model: RobotModel, q: Optional[np.ndarray] = None,
                      base_pos: Optional[np.ndarray] = None, base_rot: Optional[np.ndarray] = None):
    """World (R, x) of every link frame; used by tests and the golden generator."""
    q = np.zeros(model.n_joint_dofs) if q is None else q
    bp = model.base_pos if base_pos is None else base_pos
    br = model.base_rot if base_rot is None else base_rot
    Rs, xs = [], []
    for l in model.links:
        Rp, xp = (br, bp) if l.parent < 0 else (Rs[l.parent], xs[l.parent])
        R0 = Rp @ l.offset_rot
        x0 = xp + Rp @ l.offset_pos
        if l.jtype == JOINT_REVOLUTE:
            Rj = axisangle_to_mat(l.axis, q[l.dof])
            R = R0 @ Rj
            x = x0 + R0 @ (l.anchor - Rj @ l.anchor)
        elif l.jtype == JOINT_PRISMATIC:
            R = R0
            x = x0 + R0 @ (l.axis * q[l.dof])
        else:
            R, x = R0, x0
        Rs.append(R)
        xs.append(x)
    return Rs, xs

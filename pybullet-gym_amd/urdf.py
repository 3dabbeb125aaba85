"""URDF -> static articulated-robot tables (Atlas).

The reference loads ``atlas/atlas_description/atlas_v4_with_multisense.urdf`` with
``pybullet.loadURDF(path, basePosition, baseOrientation, useFixedBase=False)`` and no flags
(``robot_bases.py:145-164``: URDFBasedRobot, self_collision False), then walks the multibody
with ``getJointInfo`` in ``XmlBasedRobot.addToScene`` (``robot_bases.py:32-91``).  pybullet's URDF
importer (URDF2Bullet) is third-party C++ absent from /root/reference; its rules are restated
here as explicit choices [EXT, unpinned], in the same RobotModel the MJCF compiler produces:

* U1 topology: the link that is no joint's child is the base (Atlas: ``pelvis``), floating
  (useFixedBase False).  Multibody link indices follow URDF2Bullet's ComputeParentIndices: a
  depth-first pre-order from the base, each link's children in the order their joints appear
  in the file.  ``continuous`` joints are unlimited revolute joints, ``fixed`` joints fixed
  links.
* U2 frames: a link's frame is its URDF link frame (the joint frame); the joint anchor is its
  origin, the axis the joint's ``<axis>``; the base frame is the base's centre of mass (what
  getBasePositionAndOrientation reports), so the base's children are offset by -COM.
* U3 mass: the ``<inertial><mass>``; inertia: without URDF_USE_INERTIA_FROM_FILE pybullet
  recomputes it from the collision shapes -- btCompoundShape's AABB box approximation,
  I = m/12 (l_y^2 + l_z^2, ...) diagonal in the inertial frame's axes (every Atlas inertial
  frame is unrotated), as mjcf.py B3; a link without collision shapes keeps the URDF's
  ``<inertia>``.
* U4 collision: ``<box>``, ``<cylinder>`` (btCylinderShapeZ) and ``<sphere>`` shapes at their
  ``<origin>``; link friction btCollisionObject's default 0.5 (no ``<contact>`` element) times
  the floor's 0.8.  Floor contact candidates ("slots", radius 0 unless a sphere): the 8
  corners of a box, CYL_RIM_POINTS points on each cap rim of a cylinder (Bullet's
  convex-plane manifold keeps <= 4 of the deepest such points), a sphere's centre with its
  radius.
* U5 joints: ``<limit lower upper>`` -> pybullet limits (joint-limit rows when lower < upper);
  ``<limit velocity>`` -> getJointInfo's maxVelocity, which current_relative_position divides
  joint speed by (robot_bases.py:314-315); ``<dynamics damping>`` -> -d qdot per sub-step as
  mjcf.py B6; ``<limit effort>`` does not clamp TORQUE_CONTROL torques.
* U6 one robot per env (a deliberate divergence): the reference's URDFBasedRobot.reset has no
  ``doneLoading`` guard (``robot_bases.py:145-164``, unlike the MJCF robots' ``:107-116``), so
  every env reset calls ``loadURDF`` again, and from the second episode on the reference scene
  holds the earlier episodes' Atlas bodies beside the new one (``restoreState`` at
  ``gym_locomotion_envs.py:35-36`` restores the snapshot's bodies, the new body is added at the
  spawn pose and overlaps them; ``addToScene`` then rebinds parts / joints to the newest body).
  That growth of the scene is a reference artefact no learner relies on; the port models exactly
  one Atlas per env in every episode.  Atlas parity beyond the first episode is therefore
  unpinned even where the first episode's would be.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict, List, Tuple

import numpy as np

from .mjcf import (GEOM_BOX, GEOM_CYLINDER, GEOM_SPHERE, JOINT_FIXED, JOINT_PRISMATIC, JOINT_REVOLUTE, Geom,
                   Link, RobotModel)

LINK_FRICTION = 0.5   # btCollisionObject::m_friction default (URDF without <contact>)
CYL_RIM_POINTS = 6    # floor-contact points per cylinder cap rim (U4)


def rpy_to_mat(rpy) -> np.ndarray:
    """URDF origin rpy: R = Rz(yaw) Ry(pitch) Rx(roll) (fixed-axis roll, pitch, yaw)."""
    r, p, y = [float(v) for v in rpy]
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _vec(s, n=3) -> np.ndarray:
    if s is None:
        return np.zeros(n)
    return np.array([float(x) for x in s.split()], dtype=float)


def _origin(el) -> Tuple[np.ndarray, np.ndarray]:
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.zeros(3), np.eye(3)
    return _vec(o.get("xyz")), rpy_to_mat(_vec(o.get("rpy")))


def _geom(col) -> Geom:
    pos, rot = _origin(col)
    g = col.find("geometry")[0]
    if g.tag == "box":
        half = 0.5 * _vec(g.get("size"))
        return Geom("box", GEOM_BOX, 0.0, pos.copy(), pos.copy(), LINK_FRICTION, 1, 1, half=half, rot=rot)
    if g.tag == "cylinder":
        r, L = float(g.get("radius")), float(g.get("length"))
        ax = rot @ np.array([0.0, 0.0, 0.5 * L])
        return Geom("cylinder", GEOM_CYLINDER, r, pos - ax, pos + ax, LINK_FRICTION, 1, 1,
                    half=np.array([r, r, 0.5 * L]), rot=rot)
    if g.tag == "sphere":
        r = float(g.get("radius"))
        return Geom("sphere", GEOM_SPHERE, r, pos.copy(), pos.copy(), LINK_FRICTION, 1, 1)
    raise NotImplementedError(f"URDF collision geometry {g.tag}")


def geom_aabb(geoms) -> Tuple[np.ndarray, np.ndarray]:
    """AABB (link axes) of a compound of boxes / Z cylinders / spheres: |R| half extents
    (btBoxShape / btCylinderShape::getAabb), +-r for a sphere."""
    lo, hi = np.full(3, np.inf), np.full(3, -np.inf)
    for g in geoms:
        c = 0.5 * (g.p0 + g.p1)
        ext = np.full(3, g.radius) if g.kind == GEOM_SPHERE else np.abs(g.rot) @ g.half
        lo, hi = np.minimum(lo, c - ext), np.maximum(hi, c + ext)
    return lo, hi


def aabb_inertia(geoms, mass: float) -> np.ndarray:
    """U3: btCompoundShape::calculateLocalInertia (the AABB's solid box)."""
    if not geoms:
        return np.zeros((3, 3))
    lo, hi = geom_aabb(geoms)
    l = hi - lo
    return np.diag([mass / 12.0 * (l[1] ** 2 + l[2] ** 2), mass / 12.0 * (l[0] ** 2 + l[2] ** 2),
                    mass / 12.0 * (l[0] ** 2 + l[1] ** 2)])


def geom_contact_points(g: Geom) -> List[Tuple[np.ndarray, float]]:
    """U4: floor-contact candidate points (link frame) and radii of one collision shape."""
    if g.kind == GEOM_SPHERE:
        return [(g.p0.copy(), g.radius)]
    if g.kind == GEOM_BOX:
        c = g.p0
        return [(c + g.rot @ (g.half * np.array([sx, sy, sz])), 0.0)
                for sz in (-1.0, 1.0) for sy in (-1.0, 1.0) for sx in (-1.0, 1.0)]
    if g.kind == GEOM_CYLINDER:
        out = []
        for cap in (g.p0, g.p1):
            for k in range(CYL_RIM_POINTS):
                a = 2.0 * math.pi * k / CYL_RIM_POINTS
                out.append((cap + g.rot @ np.array([g.radius * math.cos(a), g.radius * math.sin(a), 0.0]), 0.0))
        return out
    raise NotImplementedError(g.kind)


def compile_urdf(path: str, robot_name: str, base_pos=(0.0, 0.0, 0.0)) -> RobotModel:
    """Compile one URDF (reference asset) into a RobotModel.  base_pos: the base COM's world
    position of the reset snapshot (Atlas: robot_specific_reset -> reset_pose([0, 0, 1]),
    robot_locomotors.py:338-340; the saved state holds it)."""
    root = ET.parse(path).getroot()
    links_el: Dict[str, ET.Element] = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    child_of = {j.find("child").get("link"): j for j in joints}
    children: Dict[str, List[ET.Element]] = {n: [] for n in links_el}
    for j in joints:  # URDF2Bullet: children in joint file order
        children[j.find("parent").get("link")].append(j)
    roots = [n for n in links_el if n not in child_of]
    assert len(roots) == 1, roots

    def inertial(name):
        el = links_el[name]
        ine = el.find("inertial")
        mass = float(ine.find("mass").get("value")) if ine is not None else 0.0
        com, crot = _origin(ine) if ine is not None else (np.zeros(3), np.eye(3))
        assert np.allclose(crot, np.eye(3)), f"{name}: rotated inertial frame"
        geoms = [_geom(c) for c in el.findall("collision")]
        if geoms or ine is None or ine.find("inertia") is None:
            return mass, com, aabb_inertia(geoms, mass), geoms
        # no collision shape (Atlas ltorso): the URDF's own inertia stands (U3)
        a = {k: float(ine.find("inertia").get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
        inert = np.array([[a["ixx"], a["ixy"], a["ixz"]], [a["ixy"], a["iyy"], a["iyz"]], [a["ixz"], a["iyz"], a["izz"]]])
        return mass, com, inert, geoms

    base = roots[0]
    bm, bcom, binert, bgeoms = inertial(base)
    shifted = lambda g, d: Geom(g.name, g.kind, g.radius, g.p0 + d, g.p1 + d, g.friction, g.contype,
                                g.conaffinity, g.mass, g.half, g.rot)
    links: List[Link] = []

    def add(j, parent_index: int, shift: np.ndarray):
        jt = j.get("type")
        child = j.find("child").get("link")
        pos, rot = _origin(j)
        axis = _vec(j.find("axis").get("xyz")) if j.find("axis") is not None else np.array([1.0, 0.0, 0.0])
        axis = axis / np.linalg.norm(axis)
        lim = j.find("limit")
        lo = float(lim.get("lower", "0")) if lim is not None else 0.0
        hi = float(lim.get("upper", "-1")) if lim is not None else -1.0
        vmax = float(lim.get("velocity", "0")) if lim is not None else 0.0
        dyn = j.find("dynamics")
        damping = float(dyn.get("damping", "0")) if dyn is not None else 0.0
        if jt in ("revolute", "continuous"):
            jtype = JOINT_REVOLUTE
        elif jt == "prismatic":
            jtype = JOINT_PRISMATIC
        elif jt == "fixed":
            jtype = JOINT_FIXED
        else:
            raise NotImplementedError(jt)
        limited = jt in ("revolute", "prismatic") and lo < hi
        m, com, inert, geoms = inertial(child)
        links.append(Link(name=child, joint_name=j.get("name"), parent=parent_index, jtype=jtype,
                          offset_pos=pos - shift, offset_rot=rot, axis=axis if jtype != JOINT_FIXED else np.zeros(3),
                          anchor=np.zeros(3), lower=lo if limited else 0.0, upper=hi if limited else -1.0,
                          limited=limited, damping=damping, mass=m, com=com, inertia=inert, geoms=geoms,
                          body=child, max_velocity=vmax))
        me = len(links) - 1
        for cj in children[child]:
            add(cj, me, np.zeros(3))

    for j in children[base]:
        add(j, -1, bcom)
    model = RobotModel(name=robot_name, floating=True, base_name=base, base_mass=bm, base_inertia=binert,
                       base_pos=np.asarray(base_pos, dtype=float), base_rot=np.eye(3),
                       base_geoms=[shifted(g, -bcom) for g in bgeoms], links=links)
    d = 0
    for l in model.links:
        if l.jtype != JOINT_FIXED:
            l.dof = d
            d += 1
    return model

"""Compiled robot tables -> ``models/<robot>.json`` and the C++ header ``csrc/models_gen.h``.

The header is the one place the HIP kernel and the CPU oracle learn a robot's
topology, mass properties, contact slots, observation layout and reward constants.
Regenerate with ``python -m pybulletgym_amd.codegen`` (needs /root/reference for the
MJCF assets); ``tests/test_models.py`` checks that the committed files are current.
"""
from __future__ import annotations

import json
import math
import os
import sys
from typing import Dict, List

import numpy as np

from . import mjcf, robots

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(HERE, "csrc", "models_gen.h")
MODEL_DIR = os.path.join(HERE, "models")
# Importer-rule overrides: a pybullet dump, when one exists, replaces the
# mjcf.py rules B3-B6 per robot without code changes.  Format (every key optional):
#   {"<robot key>": {"contact_erp": e, "floor_lateral_friction": mu_floor,
#      "links":  {"<link or base name>": {"mass": m, "local_inertia_diagonal": [ix, iy, iz],
#                                         "lateral_friction": mu}},      # getDynamicsInfo fields
#      "joints": {"<joint name>": {"damping": d, "lower": lo, "upper": hi}}}}  # getJointInfo fields
OVERRIDES = os.path.join(MODEL_DIR, "importer_overrides.json")
CONTACT_ERP_DEFAULT = 0.2  # sim_params.h PBG_CONTACT_ERP (Bullet btContactSolverInfo::m_erp)


def load_overrides(path: str = None) -> Dict:
    path = path or OVERRIDES
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        ov = json.load(f)
    return {k: v for k, v in ov.items() if not k.startswith("_")}


def apply_overrides(model: mjcf.RobotModel, ov: Dict) -> None:
    """Replace the imported mass / inertia / friction / joint damping and limits by the values
    a pybullet dump reports (getDynamicsInfo / getJointInfo), in place."""
    floor_mu = ov.get("floor_lateral_friction")
    for name, d in ov.get("links", {}).items():
        if name == model.base_name:
            if "mass" in d:
                model.base_mass = float(d["mass"])
            if "local_inertia_diagonal" in d:
                model.base_inertia = np.diag([float(x) for x in d["local_inertia_diagonal"]])
            geoms = model.base_geoms
        else:
            link = model.links[model.link_index(name)]
            if "mass" in d:
                link.mass = float(d["mass"])
            if "local_inertia_diagonal" in d:
                link.inertia = np.diag([float(x) for x in d["local_inertia_diagonal"]])
            geoms = link.geoms
        if "lateral_friction" in d:
            for g in geoms:
                g.friction = float(d["lateral_friction"])
    for name, d in ov.get("joints", {}).items():
        hits = [l for l in model.links if l.joint_name == name]
        if not hits:
            raise KeyError(f"override for unknown joint {name!r}")
        for l in hits:
            if "damping" in d:
                l.damping = float(d["damping"])
            if "lower" in d and "upper" in d:
                l.lower, l.upper = float(d["lower"]), float(d["upper"])
                l.limited = l.lower <= l.upper
    return floor_mu


def _chain_links(model: mjcf.RobotModel, li: int) -> List[int]:
    """li and its ancestors (root first)."""
    out = [li]
    out += model.ancestors(li)
    return out[::-1]


# HumanoidFlagrunHarder's cube: cube_small.urdf <lateral_friction value="1.0"/> (pybullet_data;
# envs/assets/things/cube_small.urdf), combined with the other body's friction by product [EXT]
CUBE_FRICTION = 1.0


def build_tables(spec: robots.RobotSpec, model: mjcf.RobotModel, ov: Dict = None) -> Dict:
    ov = ov or {}
    floor_mu = apply_overrides(model, ov)
    floor_mu = mjcf.FLOOR_FRICTION if floor_mu is None else float(floor_mu)
    parts, ordered, robot_body = robots.add_to_scene_order(model, spec.robot_name)
    L = model.n_links
    NJ = model.n_joint_dofs
    links = model.links
    # actions: Humanoid applies actions in motor_names order (robot_locomotors.py:185-189);
    # every other robot uses ordered_joints order (:26-29).  calc_state always reads
    # ordered_joints (:32).
    ordered_names = [links[i].joint_name for i in ordered]
    if spec.motor_order is not None:
        assert spec.motor_order == ordered_names, "Humanoid motor order == ordered_joints order"
    tip_link = -1
    if spec.kind == robots.KIND_PENDULUM and spec.alive in (robots.ALIVE_DOUBLE, robots.ALIVE_DOUBLE_MJ):
        # robot_pendula.py:72-88: slider torque 200*clip(a0); reset randomises hinge, hinge2
        # (:66-68); calc_state reads hinge, hinge2, slider and pole2's position (:81-83).
        act_links = [model.link_index("cart")]
        act_gain = [100.0 * spec.power]
        reset_dof = [links[model.link_index("pole")].dof, links[model.link_index("pole2")].dof]
        obs_links = [model.link_index("pole"), model.link_index("pole2"), model.link_index("cart")]
        tip_link = model.link_index("pole2")
    elif spec.kind == robots.KIND_PENDULUM:
        # robot_pendula.py:20-25: one action, slider torque 100*clip(a0); reset randomises
        # only the hinge (:16-17); calc_state reads hinge then slider (:28-29).
        act_links = [model.link_index("cart")]
        act_gain = [100.0]
        reset_dof = [links[model.link_index("pole")].dof]
        obs_links = [model.link_index("pole"), model.link_index("cart")]
    elif spec.kind == robots.KIND_MUJOCO_PLANAR:
        # mujoco/robot_bases.py:82-95 add_ignored_joints: the ignored root joints join
        # ordered_joints (power_coef 0, skipped by apply_action, mujoco robot_locomotors.py:26-33)
        # and are re-randomised at reset (:17-19) and read by calc_state like the others.
        all_ordered = [i for i, l in enumerate(links) if l.dof >= 0 and l.joint_name[:8] != "jointfix"]
        act_links = list(ordered)
        act_gain = [spec.power * spec.power_coef.get(links[i].joint_name, 100.0) for i in ordered]
        reset_dof = [links[i].dof for i in all_ordered]
        obs_links = all_ordered
    else:
        act_links = list(ordered)
        act_gain = [spec.power * spec.power_coef.get(links[i].joint_name, 100.0)  # robot_locomotors.py:29,
                    for i in ordered]                                             # robot_bases.py:89
        reset_dof = [links[i].dof for i in ordered]   # robot_locomotors.py:18-19
        obs_links = list(ordered)
    act_dof = [links[i].dof for i in act_links]
    obs_dof = [links[i].dof for i in obs_links]
    # joint observation scaling (robot_bases.py:306-321): MJCF joints report maxVelocity 0
    # (x0.1 revolute, x0.5 prismatic); URDF joints their <limit velocity> (urdf.py U5): 1 / maxVel
    vel_scale = [1.0 / links[i].max_velocity if links[i].max_velocity > 0 else
                 (0.1 if links[i].jtype == mjcf.JOINT_REVOLUTE else 0.5) for i in obs_links]

    dof_link = model.dof_link()
    dof = dict(
        lower=[links[i].lower for i in dof_link], upper=[links[i].upper for i in dof_link],
        limited=[int(links[i].limited) for i in dof_link], damping=[links[i].damping for i in dof_link],
        stiffness=[links[i].stiffness for i in dof_link],
        armature=[links[i].armature for i in dof_link], jtype=[links[i].jtype for i in dof_link],
        link=dof_link)

    # chain masks: bit d set if joint dof d moves link l (l itself or an ancestor)
    chain_mask = []
    for li in range(L):
        m = 0
        for a in _chain_links(model, li):
            if links[a].dof >= 0:
                m |= 1 << links[a].dof
        chain_mask.append(m)

    # link ancestor masks: bit j set if link j is link l or one of its ancestors
    anc_mask = []
    for li in range(L):
        m = 1 << li
        for a in model.ancestors(li):
            m |= 1 << a
        anc_mask.append(m)

    # floor contact slots: sphere -> centre, capsule -> both segment endpoints
    slots = []
    if spec.floor:
        def add_slots(li, geoms):
            for g in geoms:
                if g.contype == 0 and g.conaffinity == 0:
                    continue
                mu = g.friction * floor_mu
                if g.kind == mjcf.GEOM_SPHERE:
                    slots.append((li, g.p0, g.radius, mu))
                elif g.kind == mjcf.GEOM_CAPSULE:
                    slots.append((li, g.p0, g.radius, mu))
                    slots.append((li, g.p1, g.radius, mu))
                else:  # URDF box corners / cylinder rim points (urdf.py U4)
                    from . import urdf
                    for p, r in urdf.geom_contact_points(g):
                        slots.append((li, p, r, mu))
        add_slots(-1, model.base_geoms)
        for li, l in enumerate(links):
            add_slots(li, l.geoms)
        if len(slots) > 64:
            # the gang kernel reports floor contact of the first 64 slots to the feet test: the
            # feet's slots go first (the candidate order is this compiler's choice)
            fl = {model.link_index(f) for f in spec.foot_list}
            slots = [x for x in slots if x[0] in fl] + [x for x in slots if x[0] not in fl]
            assert sum(1 for x in slots if x[0] in fl) <= 64
    # self-collision pairs (Humanoid): non-ancestor link pairs, MuJoCo contype/conaffinity rule
    pairs = []
    if spec.self_collision and spec.floor:
        glist = [(li, g) for li, l in enumerate(links) for g in l.geoms]
        for a in range(len(glist)):
            for b in range(a + 1, len(glist)):
                la, ga = glist[a]
                lb, gb = glist[b]
                if la == lb or la in model.ancestors(lb) or lb in model.ancestors(la):
                    continue
                if not ((ga.contype & gb.conaffinity) or (gb.contype & ga.conaffinity)):
                    continue
                pairs.append((la, ga, lb, gb))

    # unique geoms referenced by pairs (for the kernel's per-geom world endpoints)
    pgeoms = []
    def gid(li, g):
        for k, (l2, g2) in enumerate(pgeoms):
            if l2 == li and g2 is g:
                return k
        pgeoms.append((li, g))
        return len(pgeoms) - 1
    pair_ga = [gid(p[0], p[1]) for p in pairs]
    pair_gb = [gid(p[2], p[3]) for p in pairs]

    # HumanoidFlagrunHarder: every collision geom of the robot against the cube (a separate
    # body: pybullet's default collision filter lets it hit all links), sphere p0 == p1
    cgeoms = []
    if spec.harder:
        for li, geoms in [(-1, model.base_geoms)] + [(li, l.geoms) for li, l in enumerate(links)]:
            for g in geoms:
                if g.contype == 0 and g.conaffinity == 0:
                    continue
                cgeoms.append((li, g))

    feet = [model.link_index(f) for f in spec.foot_list]
    # Atlas alive_bonus (robot_locomotors.py:313-324): the head part's height and the knees'
    # relative positions (their obs joint indices)
    head_link = model.link_index(spec.head) if spec.head else -1
    knee_obs = [ordered_names.index(k) for k in spec.knees] if spec.knees else [-1, -1]
    inertia6 = lambda I: [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]
    t = dict(
        key=spec.key, env_id=spec.env_id, kind=spec.kind, floating=int(model.floating),
        NL=L, NJ=NJ, NDOF=NJ + (6 if model.floating else 0), NA=len(act_dof), NO=len(obs_dof),
        NR=len(reset_dof), NF=len(feet),
        NP=len(parts), NS=len(slots), NPAIR=len(pairs), OBS=spec.obs_dim,
        alive=spec.alive, power=spec.power, electricity_cost=spec.electricity_cost,
        stall_torque_cost=spec.stall_torque_cost, joints_at_limit_cost=spec.joints_at_limit_cost,
        initial_z_fixed=(spec.initial_z if spec.initial_z is not None else float("nan")),
        dt_sub=spec.timestep, substeps=spec.frame_skip, floor=int(spec.floor),
        max_episode_steps=spec.max_episode_steps,
        base_mass=model.base_mass, base_inertia=inertia6(model.base_inertia),
        base_pos=list(model.base_pos), base_quat=list(mjcf.mat_to_quat_xyzw(model.base_rot)),
        link_name=[l.name for l in links], link_parent=[l.parent for l in links],
        link_jtype=[l.jtype for l in links], link_dof=[l.dof for l in links],
        link_offset_pos=[list(l.offset_pos) for l in links],
        link_offset_quat=[list(mjcf.mat_to_quat_xyzw(l.offset_rot)) for l in links],
        link_axis=[list(l.axis) for l in links], link_anchor=[list(l.anchor) for l in links],
        link_mass=[l.mass for l in links], link_com=[list(l.com) for l in links],
        link_inertia=[inertia6(l.inertia) for l in links], link_chain_mask=chain_mask,
        link_anc_mask=anc_mask,
        dof_lower=dof["lower"], dof_upper=dof["upper"], dof_limited=dof["limited"],
        dof_damping=dof["damping"], dof_stiffness=dof["stiffness"], dof_armature=dof["armature"], dof_jtype=dof["jtype"],
        dof_link=dof["link"],
        act_dof=act_dof, act_gain=act_gain, obs_dof=obs_dof, obs_vel_scale=vel_scale,
        reset_dof=reset_dof, reset_offset=[spec.reset_offset if i == 0 else 0.0 for i in range(len(reset_dof))],
        tip_link=tip_link, flagrun=int(spec.flagrun), power_cost=spec.power_cost, qvel_clip=spec.qvel_clip,
        head_link=head_link, knee_obs=knee_obs, link_max_velocity=[l.max_velocity for l in links],
        act_joint_names=ordered_names,
        part_names=list(parts.keys()), part_link=list(parts.values()), robot_body=robot_body,
        foot_link=feet,
        slot_link=[s[0] for s in slots], slot_point=[list(s[1]) for s in slots],
        slot_radius=[s[2] for s in slots], slot_mu=[s[3] for s in slots],
        pair_link_a=[p[0] for p in pairs], pair_link_b=[p[2] for p in pairs],
        pair_a0=[list(p[1].p0) for p in pairs], pair_a1=[list(p[1].p1) for p in pairs],
        pair_b0=[list(p[3].p0) for p in pairs], pair_b1=[list(p[3].p1) for p in pairs],
        pair_ra=[p[1].radius for p in pairs], pair_rb=[p[3].radius for p in pairs],
        pair_mu=[p[1].friction * p[3].friction for p in pairs],
        NG=len(pgeoms), geom_link=[g[0] for g in pgeoms], geom_p0=[list(g[1].p0) for g in pgeoms],
        geom_p1=[list(g[1].p1) for g in pgeoms], geom_r=[g[1].radius for g in pgeoms],
        pair_ga=pair_ga, pair_gb=pair_gb,
        harder=int(spec.harder), NCG=len(cgeoms), cgeom_link=[g[0] for g in cgeoms],
        cgeom_p0=[list(g[1].p0) for g in cgeoms], cgeom_p1=[list(g[1].p1) for g in cgeoms],
        cgeom_r=[g[1].radius for g in cgeoms], cgeom_mu=[g[1].friction * CUBE_FRICTION for g in cgeoms],
        cube_floor_mu=(CUBE_FRICTION * floor_mu if spec.harder else 0.0),
        contact_erp=float(ov.get("contact_erp", CONTACT_ERP_DEFAULT)),
        # robot-floor material, Bullet's btManifoldResult combiners: restitution r_a r_b; spinning
        # and rolling friction s_a mu_b + mu_a s_b (the floor has none of its own: s_b = 0)
        restitution=spec.restitution * mjcf.FLOOR_RESTITUTION,
        spin_mu=spec.spinning_friction * floor_mu, roll_mu=spec.rolling_friction * floor_mu,
    )
    return t


def compile_all(asset_dir: str = None, overrides: Dict = None) -> Dict[str, Dict]:
    """overrides: {robot key: override dict} (default: models/importer_overrides.json if present)."""
    asset_dir = asset_dir or robots.reference_asset_dir()
    overrides = load_overrides() if overrides is None else overrides
    out = {}
    for key, spec in robots.SPECS.items():
        model = robots.compile_model(spec, asset_dir)
        out[key] = build_tables(spec, model, overrides.get(key))
    return out


# ----------------------------------------------------------------------------- emit C++
def _num(v) -> str:
    v = float(v)
    if math.isnan(v):
        return "__builtin_nan(\"\")"
    r = repr(v)
    if "e" not in r and "." not in r and "inf" not in r:
        r += ".0"
    return r


def _arr1(name, ctype, vals, n=None):
    vals = list(vals)
    n = max(1, len(vals)) if n is None else n
    if not vals:
        vals = [0]
    fmt = _num if ctype == "double" else (lambda v: str(int(v)))
    return f"  static constexpr {ctype} {name}[{n}] = {{{', '.join(fmt(v) for v in vals)}}};"


def _arr2(name, ctype, rows, w):
    rows = list(rows)
    n = max(1, len(rows))
    if not rows:
        rows = [[0] * w]
    body = ", ".join("{" + ", ".join(_num(v) for v in r) + "}" for r in rows)
    return f"  static constexpr {ctype} {name}[{n}][{w}] = {{{body}}};"


def emit_struct(t: Dict) -> str:
    cls = STRUCTS[t["key"]]
    L = [f"// {t['env_id']}: generated by pybulletgym_amd.codegen from the reference MJCF asset",
         f"struct {cls} {{",
         f"  static constexpr int robot_id = {ROBOT_IDS[t['key']]};",
         f"  static constexpr int kind = {t['kind']};",
         f"  static constexpr bool floating = {'true' if t['floating'] else 'false'};"]
    for k in ("NL", "NJ", "NDOF", "NA", "NO", "NR", "NF", "NP", "NS", "NPAIR", "NG", "OBS", "alive", "substeps",
              "floor", "max_episode_steps", "robot_body", "tip_link", "flagrun", "harder", "NCG", "head_link"):
        L.append(f"  static constexpr int {k} = {int(t[k])};")
    for k in ("power", "electricity_cost", "stall_torque_cost", "joints_at_limit_cost",
              "initial_z_fixed", "dt_sub", "base_mass", "power_cost", "qvel_clip", "contact_erp", "cube_floor_mu",
              "restitution", "spin_mu", "roll_mu"):
        L.append(f"  static constexpr double {k} = {_num(t[k])};")
    L.append(_arr1("base_inertia", "double", t["base_inertia"]))
    L.append(_arr1("base_pos", "double", t["base_pos"]))
    L.append(_arr1("base_quat", "double", t["base_quat"]))
    for k in ("link_parent", "link_jtype", "link_dof"):
        L.append(_arr1(k, "int", t[k]))
    L.append(_arr1("link_chain_mask", "unsigned", t["link_chain_mask"]))
    L.append(_arr1("link_anc_mask", "unsigned", t["link_anc_mask"]))
    for k in ("link_offset_pos", "link_axis", "link_anchor", "link_com"):
        L.append(_arr2(k, "double", t[k], 3))
    L.append(_arr2("link_offset_quat", "double", t["link_offset_quat"], 4))
    L.append(_arr2("link_inertia", "double", t["link_inertia"], 6))
    L.append(_arr1("link_mass", "double", t["link_mass"]))
    for k in ("dof_lower", "dof_upper", "dof_damping", "dof_stiffness", "dof_armature"):
        L.append(_arr1(k, "double", t[k]))
    for k in ("dof_limited", "dof_jtype", "dof_link"):
        L.append(_arr1(k, "int", t[k]))
    L.append(_arr1("act_dof", "int", t["act_dof"]))
    L.append(_arr1("act_gain", "double", t["act_gain"]))
    L.append(_arr1("obs_dof", "int", t["obs_dof"]))
    L.append(_arr1("obs_vel_scale", "double", t["obs_vel_scale"]))
    L.append(_arr1("reset_dof", "int", t["reset_dof"]))
    L.append(_arr1("reset_offset", "double", t["reset_offset"]))
    L.append(_arr1("part_link", "int", t["part_link"]))
    L.append(_arr1("foot_link", "int", t["foot_link"]))
    L.append(_arr1("knee_obs", "int", t["knee_obs"]))
    L.append(_arr1("slot_link", "int", t["slot_link"]))
    L.append(_arr2("slot_point", "double", t["slot_point"], 3))
    L.append(_arr1("slot_radius", "double", t["slot_radius"]))
    L.append(_arr1("slot_mu", "double", t["slot_mu"]))
    L.append(_arr1("pair_link_a", "int", t["pair_link_a"]))
    L.append(_arr1("pair_link_b", "int", t["pair_link_b"]))
    for k in ("pair_a0", "pair_a1", "pair_b0", "pair_b1"):
        L.append(_arr2(k, "double", t[k], 3))
    for k in ("pair_ra", "pair_rb", "pair_mu"):
        L.append(_arr1(k, "double", t[k]))
    L.append(_arr1("pair_ga", "int", t["pair_ga"]))
    L.append(_arr1("pair_gb", "int", t["pair_gb"]))
    L.append(_arr1("geom_link", "int", t["geom_link"]))
    L.append(_arr2("geom_p0", "double", t["geom_p0"], 3))
    L.append(_arr2("geom_p1", "double", t["geom_p1"], 3))
    L.append(_arr1("geom_r", "double", t["geom_r"]))
    L.append(_arr1("cgeom_link", "int", t["cgeom_link"]))
    L.append(_arr2("cgeom_p0", "double", t["cgeom_p0"], 3))
    L.append(_arr2("cgeom_p1", "double", t["cgeom_p1"], 3))
    L.append(_arr1("cgeom_r", "double", t["cgeom_r"]))
    L.append(_arr1("cgeom_mu", "double", t["cgeom_mu"]))
    L.append("};")
    return "\n".join(L)


ROBOT_IDS = {"pendulum": 0, "hopper": 1, "halfcheetah": 2, "ant": 3, "humanoid": 4, "walker2d": 5,
             "pendulum_swingup": 6, "double_pendulum": 7, "humanoid_flagrun": 8, "hopper_mujoco": 9,
             "walker2d_mujoco": 10, "halfcheetah_mujoco": 11, "ant_mujoco": 12, "humanoid_mujoco": 13,
             "double_pendulum_mujoco": 14, "humanoid_flagrun_harder": 15, "atlas": 16}
STRUCTS = {"pendulum": "Pendulum", "hopper": "Hopper", "halfcheetah": "HalfCheetah", "ant": "Ant",
           "humanoid": "Humanoid", "walker2d": "Walker2D", "pendulum_swingup": "PendulumSwingup",
           "double_pendulum": "DoublePendulum", "humanoid_flagrun": "HumanoidFlagrun",
           "hopper_mujoco": "HopperMuJoCo", "walker2d_mujoco": "Walker2DMuJoCo",
           "halfcheetah_mujoco": "HalfCheetahMuJoCo", "ant_mujoco": "AntMuJoCo", "humanoid_mujoco": "HumanoidMuJoCo",
           "double_pendulum_mujoco": "DoublePendulumMuJoCo", "humanoid_flagrun_harder": "HumanoidFlagrunHarder",
           "atlas": "Atlas"}


def emit_header(tables: Dict[str, Dict]) -> str:
    out = ["// GENERATED FILE - do not edit.  python -m pybulletgym_amd.codegen",
           "// Per-robot static tables compiled from the reference's MJCF assets",
           "// (pybulletgym/envs/assets/mjcf/*.xml) under the import rules in mjcf.py.",
           "#pragma once", "", "namespace pbg_models {", ""]
    for key in ROBOT_IDS:
        out.append(emit_struct(tables[key]))
        out.append("")
    out.append("}  // namespace pbg_models")
    return "\n".join(out) + "\n"


def _jsonable(t):
    return {k: (v if not isinstance(v, float) or not math.isnan(v) else None) for k, v in t.items()}


def write_all(tables=None):
    tables = tables or compile_all()
    os.makedirs(MODEL_DIR, exist_ok=True)
    for key, t in tables.items():
        with open(os.path.join(MODEL_DIR, f"{key}.json"), "w") as f:
            json.dump(_jsonable(t), f, indent=1, default=float)
    with open(HEADER, "w") as f:
        f.write(emit_header(tables))


def load_tables(key: str) -> Dict:
    with open(os.path.join(MODEL_DIR, f"{key}.json")) as f:
        t = json.load(f)
    if t.get("initial_z_fixed") is None:
        t["initial_z_fixed"] = float("nan")
    return t


if __name__ == "__main__":
    write_all()
    print("wrote", HEADER, "and", MODEL_DIR, file=sys.stderr)

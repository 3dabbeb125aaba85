"""Physics-rule study: score the reference's pretrained policies on the CPU oracle under
solver/contact rule variants (oracle pbg_oracle_set_physics) and importer-rule variants (link
masses / COMs / inertias recompiled from the reference assets and pushed with
pbg_oracle_set_link_dynamics).  DESIGN.md section 2 records the tables this prints.  Test
infrastructure only (imports the oracle; the importer variants need /root/reference).

  python tools/physics_rules.py [variant ...]     # default: every variant below
  PBG_RULE_EPISODES=64 PBG_RULE_ENVS=Walker2DPyBulletEnv-v0,AtlasPyBulletEnv-v0 python tools/physics_rules.py ...

A variant is a name below, or `k=v,k=v` over KEYS, with the importer switches `inertia_margin=m`
and `mass_first=1` allowed among them.
"""
import copy
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import oracle  # noqa: E402
import policies  # noqa: E402

# pbg_oracle.cpp OPT_* in order (the last four: the scene's gravity / dt / sub-steps, then the
# round-4 torque-timing switch)
KEYS = ["contact_erp", "deep_erp", "deep_thr", "deep_mode", "limit_mode", "damp_mode", "fric_mode", "warm",
        "warm_fric", "limit_erp", "iters", "sep_mode", "slop", "sep_abs", "lim_sep_abs",
        "springs", "roll_mu", "spin_mu", "lim_deep_mode", "limit_cfm", "contact_cfm", "contact_thr", "margin",
        "self_collision", "gravity", "dt", "substeps", "torque_substeps", "max_coord_vel"]
DEFAULT = [-1.0, -1.0, -0.04, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.2, 5.0, 0.0, 0.0, 1.0, 1.0,
           1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.02, 0.0, 1.0, 9.8, -1.0, -1.0, -1.0, 100.0]
# importer switches (not oracle options): recompiled link dynamics; joint damping with the MJCF
# <default> inherited (round 5)
IMPORTER_KEYS = ("inertia_margin", "mass_first", "capsule_margin", "default_damping")
VARIANTS = {
    "current": {},
    "erp0.9": {"contact_erp": 0.9},
    "deep0.9": {"deep_erp": 0.9},
    "deep_nopos": {"deep_mode": 1.0},
    "limit_violated_only": {"limit_mode": 1.0},
    "damp_once": {"damp_mode": 1.0},
    "cone": {"fric_mode": 1.0},
    "one_dir": {"fric_mode": 2.0},
    "warm0.85": {"warm": 0.85},
    "warm0.85_fric": {"warm": 0.85, "warm_fric": 1.0},
    "warm0.1": {"warm": 0.1},
    "no_sep_rows": {"sep_mode": 1.0},
    "relative_sep_rows (round 1)": {"sep_abs": 0.0, "lim_sep_abs": 0.0},
    "relative_sep_limit_rows": {"lim_sep_abs": 0.0},
    # round 3: importer / solver hypotheses not scored before
    # MJCF joint stiffness as a spring to q = 0 (adopted in round 3, mjcf.py B7; "no_springs" is the
    # round-2 rule set)
    "no_springs": {"springs": 0.0},
    "roll0.08": {"roll_mu": 0.08},  # MJCF friction[2] 0.1 x floor 0.8 (btManifoldResult rolling combine)
    "spin0.08": {"spin_mu": 0.08},  # MJCF friction[1] 0.1 x floor 0.8
    "roll+spin0.08": {"roll_mu": 0.08, "spin_mu": 0.08},
    "roll0.0008": {"roll_mu": 0.0008},
    "limit_erp0.9": {"limit_erp": 0.9},
    "limit_deep_velocity_only": {"lim_deep_mode": 1.0},
    "limit_deep_erp0.9": {"lim_deep_mode": 2.0},
    "limit_cfm0.01": {"limit_cfm": 0.01},
    "limit_cfm1": {"limit_cfm": 1.0},
    "contact_cfm0.01": {"contact_cfm": 0.01},
    "contact_thr0.01": {"contact_thr": 0.01},
    "contact_thr0": {"contact_thr": 0.0},
    "margin0.01": {"margin": 0.01},
    "no_self_collision": {"self_collision": 0.0},
    # round 4: the "swing dynamics" hypotheses, alone and crossed
    # (i) apply_action's torques only in the first of the frame_skip sub-steps (Bullet clears a
    #     multibody's applied joint torques after every internal step) [EXT, SURVEY B1]
    "torque_first": {"torque_substeps": 1.0},
    # (ii) the compound AABB of the inertia grown by Bullet's default convex margin 0.04 per side
    "inertia_margin0.04": {"inertia_margin": 0.04},
    "inertia_margin0.02": {"inertia_margin": 0.02},
    # (iii) a multi-joint MJCF body's mass, COM and inertia on the FIRST link of its dummy chain
    #      (mjcf.py B2 puts them on the last, with the geoms)
    "mass_first": {"mass_first": 1.0},
    # (ii') per shape: each capsule's AABB grown by its radius (its collision margin) per side
    "capsule_margin_r": {"capsule_margin": 1.0},
    "torque_first+margin0.04": {"torque_substeps": 1.0, "inertia_margin": 0.04},
    "torque_first+mass_first": {"torque_substeps": 1.0, "mass_first": 1.0},
    "margin0.04+mass_first": {"inertia_margin": 0.04, "mass_first": 1.0},
    "torque_first+margin0.04+mass_first": {"torque_substeps": 1.0, "inertia_margin": 0.04, "mass_first": 1.0},
    # round 5: contact-free rules scored on the pendulum family first
    "default_damping": {"default_damping": 1.0},
    "max_coord_vel1000": {"max_coord_vel": 1000.0},
    "max_coord_vel10": {"max_coord_vel": 10.0},
    "margin0.04+default_damping": {"inertia_margin": 0.04, "default_damping": 1.0},
}
PENDULUMS = ["InvertedPendulumPyBulletEnv-v0", "InvertedPendulumSwingupPyBulletEnv-v0",
             "InvertedDoublePendulumPyBulletEnv-v0"]
ENVS = ["HopperPyBulletEnv-v0", "Walker2DPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0", "AntPyBulletEnv-v0",
        "HumanoidPyBulletEnv-v0", "HumanoidFlagrunPyBulletEnv-v0", "InvertedDoublePendulumPyBulletEnv-v0",
        "HumanoidFlagrunHarderPyBulletEnv-v0", "AtlasPyBulletEnv-v0"]
SHORT = {"HopperPyBulletEnv-v0": "Hopper", "Walker2DPyBulletEnv-v0": "Walker", "HalfCheetahPyBulletEnv-v0": "Cheetah",
         "AntPyBulletEnv-v0": "Ant", "HumanoidPyBulletEnv-v0": "Humanoid", "HumanoidFlagrunPyBulletEnv-v0": "Flagrun",
         "InvertedDoublePendulumPyBulletEnv-v0": "DblPend", "HumanoidFlagrunHarderPyBulletEnv-v0": "Harder",
         "AtlasPyBulletEnv-v0": "Atlas"}
SHORT.update({"InvertedPendulumPyBulletEnv-v0": "Pendulum", "InvertedPendulumSwingupPyBulletEnv-v0": "Swingup"})


def set_physics(over):
    v = list(DEFAULT)
    for k, x in over.items():
        if k in IMPORTER_KEYS:
            continue
        v[KEYS.index(k)] = x
    arr = np.array(v, dtype=np.float64)
    L = oracle.lib()
    L.pbg_oracle_set_physics.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.pbg_oracle_set_physics(arr.ctypes.data_as(ctypes.c_void_p), len(v))


def importer_tables(env_id, margin=0.0, mass_first=False, capsule_margin=0.0, default_damping=False):
    """The robot's compiled tables under the importer variant (mjcf.py B2/B3, urdf.py U3).
    margin: the compound AABB grown by `margin` per side; capsule_margin: each capsule's AABB grown
    by capsule_margin x its radius per side before the union (a btCapsuleShape's collision margin is
    its radius; whether its getAabb adds the margin on top of the radius is the question)."""
    from pybulletgym_amd import codegen, mjcf, robots, urdf
    spec = next(s for s in robots.SPECS.values() if s.env_id == env_id)
    saved = (mjcf.bullet_compound_inertia, urdf.aabb_inertia, mjcf.collision_aabb, mjcf.INHERIT_DEFAULT_DAMPING)
    orig_aabb = mjcf.collision_aabb

    def capsule_aabb(geoms):
        lo, hi = orig_aabb(geoms)
        for g in geoms:
            if g.kind == mjcf.GEOM_CAPSULE:
                glo, ghi = orig_aabb([g])
                lo, hi = np.minimum(lo, glo - capsule_margin * g.radius), np.maximum(hi, ghi + capsule_margin * g.radius)
        return lo, hi

    def grown(fn_aabb):
        def inertia(geoms, mass):
            if not geoms:
                return np.zeros((3, 3))
            lo, hi = fn_aabb(geoms)
            lo, hi = lo - margin, hi + margin
            l = hi - lo
            return np.diag([mass / 12.0 * (l[1] ** 2 + l[2] ** 2), mass / 12.0 * (l[0] ** 2 + l[2] ** 2),
                            mass / 12.0 * (l[0] ** 2 + l[1] ** 2)])
        return inertia
    try:
        mjcf.INHERIT_DEFAULT_DAMPING = bool(default_damping)
        if capsule_margin:
            mjcf.collision_aabb = capsule_aabb
        if margin or capsule_margin:
            mjcf.bullet_compound_inertia = grown(mjcf.collision_aabb)
            urdf.aabb_inertia = grown(urdf.geom_aabb)
        model = robots.compile_model(spec)
    finally:
        mjcf.bullet_compound_inertia, urdf.aabb_inertia, mjcf.collision_aabb, mjcf.INHERIT_DEFAULT_DAMPING = saved
    if mass_first:
        # links of one MJCF body: its dummies then the real link (mjcf.py add_body), same frame
        by_body = {}
        for i, l in enumerate(model.links):
            by_body.setdefault(l.body, []).append(i)
        for idx in by_body.values():
            if len(idx) < 2:
                continue
            first, real = model.links[idx[0]], model.links[idx[-1]]
            first.mass, first.com, first.inertia = real.mass, real.com.copy(), real.inertia.copy()
            real.mass, real.com, real.inertia = 0.0, np.zeros(3), np.zeros((3, 3))
    return codegen.build_tables(spec, model, codegen.load_overrides().get(spec.key))


def set_importer(env_id, over):
    L = oracle.lib()
    L.pbg_oracle_set_link_dynamics.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_double, ctypes.c_void_p]
    rid = oracle.robot_id(env_id)
    margin, mass_first = float(over.get("inertia_margin", 0.0)), bool(over.get("mass_first", 0.0))
    cmargin = float(over.get("capsule_margin", 0.0))
    ddamp = bool(over.get("default_damping", 0.0))
    L.pbg_oracle_set_dof_damping.argtypes = [ctypes.c_int, ctypes.c_void_p]
    if not margin and not mass_first and not cmargin and not ddamp:
        L.pbg_oracle_set_link_dynamics(rid, None, None, None, 0.0, None)
        L.pbg_oracle_set_dof_damping(rid, None)
        return
    t = importer_tables(env_id, margin, mass_first, cmargin, ddamp)
    damp = np.ascontiguousarray(t["dof_damping"], dtype=np.float64)
    L.pbg_oracle_set_dof_damping(rid, damp.ctypes.data)
    p = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    mass, com, inertia, bi = p(t["link_mass"]), p(t["link_com"]), p(t["link_inertia"]), p(t["base_inertia"])
    _keep = (mass, com, inertia, bi)
    L.pbg_oracle_set_link_dynamics(rid, mass.ctypes.data, com.ctypes.data, inertia.ctypes.data, float(t["base_mass"]),
                                   bi.ctypes.data)
    del _keep


def score(over, envs=None, n=int(os.environ.get("PBG_RULE_EPISODES", "16"))):
    envs = envs or ENVS
    set_physics(over)
    out = {}
    for env_id in envs:
        set_importer(env_id, over)
        ret, ln = policies.episode_returns_oracle(env_id, n, seed=0)
        out[env_id] = (ret.mean(), ln.mean())
        set_importer(env_id, {})
    set_physics({})
    return out


def parse(spec):
    """name or k=v,k=v"""
    if spec in VARIANTS or spec.startswith("relative_sep_rows"):
        spec = "relative_sep_rows (round 1)" if spec.startswith("relative_sep_rows") else spec
        return spec, VARIANTS[spec]
    d = {}
    for kv in spec.split(","):
        k, v = kv.split("=")
        d[k] = float(v)
    return spec, d


if __name__ == "__main__":
    specs = sys.argv[1:] or list(VARIANTS)
    envs = os.environ.get("PBG_RULE_ENVS", "").split(",") if os.environ.get("PBG_RULE_ENVS") else ENVS
    if envs == ["pendulums"]:
        envs = PENDULUMS
    print(f"{'variant':38s}" + "".join(f"{SHORT[e]:>16s}" for e in envs), flush=True)
    for sp in specs:
        name, over = parse(sp)
        sc = score(over, envs)
        print(f"{name:38s}" + "".join(f"{sc[e][0]:9.0f} ({sc[e][1]:4.0f})" for e in envs), flush=True)

"""Physics-rule study: score the reference's pretrained policies on the CPU oracle under
solver/contact rule variants (oracle pbg_oracle_set_physics).  DESIGN.md section 2 records
the table this prints.  Test infrastructure only (imports the oracle).

  python tools/physics_rules.py [variant ...]     # default: every variant below
"""
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

KEYS = ["contact_erp", "deep_erp", "deep_thr", "deep_mode", "limit_mode", "damp_mode", "fric_mode", "warm",
        "warm_fric", "limit_erp", "iters", "sep_mode", "slop", "sep_abs", "lim_sep_abs",
        "springs", "roll_mu", "spin_mu", "lim_deep_mode", "limit_cfm", "contact_cfm", "contact_thr", "margin",
        "self_collision"]
DEFAULT = [-1.0, -1.0, -0.04, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.2, 5.0, 0.0, 0.0, 1.0, 1.0,
           1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.02, 0.0, 1.0]
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
}
ENVS = ["HopperPyBulletEnv-v0", "Walker2DPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0", "AntPyBulletEnv-v0",
        "HumanoidPyBulletEnv-v0", "HumanoidFlagrunPyBulletEnv-v0", "InvertedDoublePendulumPyBulletEnv-v0"]


def set_physics(over):
    v = list(DEFAULT)
    for k, x in over.items():
        v[KEYS.index(k)] = x
    arr = np.array(v, dtype=np.float64)
    L = oracle.lib()
    L.pbg_oracle_set_physics.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.pbg_oracle_set_physics(arr.ctypes.data_as(ctypes.c_void_p), len(v))


def score(over, envs=ENVS, n=int(os.environ.get("PBG_RULE_EPISODES", "16"))):
    set_physics(over)
    out = {}
    for env_id in envs:
        ret, ln = policies.episode_returns_oracle(env_id, n, seed=0)
        out[env_id] = (ret.mean(), ln.mean())
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
    short = ["Hopper", "Walker", "Cheetah", "Ant", "Humanoid", "Flagrun", "DblPend"]
    print(f"{'variant':34s}" + "".join(f"{s:>16s}" for s in short))
    for sp in specs:
        name, over = parse(sp)
        sc = score(over)
        print(f"{name:34s}" + "".join(f"{sc[e][0]:9.0f} ({sc[e][1]:4.0f})" for e in ENVS), flush=True)

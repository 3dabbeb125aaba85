"""Joint fit of the contact-free dynamics on the double pendulum.

The reference's pretrained InvertedDoublePendulum policy (examples/roboschool-weights/
enjoy_TF_InvertedDoublePendulumPyBulletEnv_v0_2017jul.py) scores 9,100+ on pybullet (the
registry's reward threshold, /root/reference/pybulletgym/envs/__init__.py:12-15); on the oracle's
physics it scores 7,558 (512 episodes).  The env has no contacts (gym_pendulum_envs.py:52-86:
SingleRobotEmptyScene, cart slider + two hinges, robot_pendula.py:58-88), so the gap lies in the
masses, the inertias, the joint damping or the integration of the 16.5 ms step.  Earlier rounds
toggled one rule at a time; this searches them jointly:

  cart mass scale, pole mass scale (both poles), inertia: the compound-AABB margin (Bullet's convex
  margin, mjcf.py B3) and a scale on top, hinge / slider damping, and the integration: k sub-steps of
  16.5 / k ms per env step (k = 1 is pybullet's numSubSteps = frame_skip = 1).

Stage 1 screens a grid at PBG_FIT_SCREEN episodes (default 128), stage 2 re-scores the best
PBG_FIT_TOP cells at 512 episodes.  Output: one line per cell, then the surface summary (best return
per knob value, the others maximised over).  Test infrastructure only (imports the oracle; the
importer tables need /root/reference).

  python tools/pendulum_fit.py > profiles/r06_pendulum_fit.txt
"""
import itertools
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import physics_rules as pr  # noqa: E402
import policies  # noqa: E402  (physics_rules put tests/ on the path)
import oracle  # noqa: E402

ENV = "InvertedDoublePendulumPyBulletEnv-v0"
THRESHOLD = 9100.0
CART = [0.25, 0.5, 1.0, 2.0, 4.0]
POLE = [0.5, 0.75, 1.0, 1.25, 1.5, 2.0]
MARGIN = [0.0, 0.04, 0.1]
ISCALE = [0.5, 0.75, 1.0, 1.5, 2.0, 3.0]
DAMP = [0.0, 0.01, 0.05, 0.1]
SUBSTEPS = [1, 2, 4, 8]
SCREEN = int(os.environ.get("PBG_FIT_SCREEN", "128"))
TOP = int(os.environ.get("PBG_FIT_TOP", "20"))
THREADS = int(os.environ.get("PBG_FIT_THREADS", "6"))

_TABLES = {}


def tables(margin):
    if margin not in _TABLES:
        _TABLES[margin] = pr.importer_tables(ENV, margin=margin)
    return _TABLES[margin]


def apply(cart, pole, margin, iscale, damp, k):
    """Push the variant's link dynamics, damping and integration into the oracle."""
    t = tables(margin)
    L = oracle.lib()
    rid = oracle.robot_id(ENV)
    mass = np.array(t["link_mass"], dtype=np.float64)
    inertia = np.array(t["link_inertia"], dtype=np.float64)
    # link 0 is the cart (slider), then the two poles (mjcf.py link order; checked below)
    scale = np.array([cart] + [pole] * (len(mass) - 1))
    mass = mass * scale
    inertia = inertia * (scale * iscale)[:, None]  # inertia ~ mass x (size)^2
    com = np.ascontiguousarray(t["link_com"], dtype=np.float64)
    bi = np.ascontiguousarray(t["base_inertia"], dtype=np.float64)
    mass, inertia = np.ascontiguousarray(mass), np.ascontiguousarray(inertia)
    L.pbg_oracle_set_link_dynamics.argtypes = [pr.ctypes.c_int] + [pr.ctypes.c_void_p] * 3 + \
        [pr.ctypes.c_double, pr.ctypes.c_void_p]
    L.pbg_oracle_set_link_dynamics(rid, mass.ctypes.data, com.ctypes.data, inertia.ctypes.data, float(t["base_mass"]),
                                   bi.ctypes.data)
    d = np.ascontiguousarray(np.full(len(t["dof_damping"]), damp, dtype=np.float64))
    L.pbg_oracle_set_dof_damping.argtypes = [pr.ctypes.c_int, pr.ctypes.c_void_p]
    L.pbg_oracle_set_dof_damping(rid, d.ctypes.data)
    pr.set_physics({"dt": 0.0165 / k, "substeps": float(k)} if k != 1 else {})
    return (mass, inertia, com, bi, d)  # keep the arrays alive while the oracle reads them


def reset_all():
    L = oracle.lib()
    rid = oracle.robot_id(ENV)
    L.pbg_oracle_set_link_dynamics(rid, None, None, None, 0.0, None)
    L.pbg_oracle_set_dof_damping(rid, None)
    pr.set_physics({})


def score(cell, n):
    keep = apply(*cell)
    ret, ln = policies.episode_returns_oracle(ENV, n, seed=0, nthreads=THREADS)
    del keep
    reset_all()
    return float(ret.mean()), float(ln.mean()), float(ret.std(ddof=1) / np.sqrt(n))


def main():
    t = tables(0.0)
    print(f"# {ENV}: link masses {np.round(t['link_mass'], 3).tolist()} (cart, pole, pole2), "
          f"dof damping {t['dof_damping']}, threshold {THRESHOLD:.0f}", flush=True)
    base = score((1.0, 1.0, 0.0, 1.0, 0.0, 1), 512)
    print(f"# adopted rule set, 512 episodes: return {base[0]:.0f} +- {base[2]:.0f}, length {base[1]:.0f}", flush=True)
    cells = list(itertools.product(CART, POLE, MARGIN, ISCALE, DAMP, SUBSTEPS))
    print(f"# stage 1: {len(cells)} cells x {SCREEN} episodes", flush=True)
    print("# cart  pole  margin iscale damp  k   return  (se)  length", flush=True)
    res = []
    t0 = time.time()
    for i, c in enumerate(cells):
        m, ln, se = score(c, SCREEN)
        res.append((m, c, ln, se))
        print(f"{c[0]:5.2f} {c[1]:5.2f} {c[2]:6.2f} {c[3]:6.2f} {c[4]:5.2f} {c[5]:2d} {m:8.0f} ({se:4.0f}) {ln:6.0f}",
              flush=True)
        if i % 500 == 499:
            print(f"# {i + 1}/{len(cells)} cells, {time.time() - t0:.0f} s", flush=True)
    res.sort(key=lambda r: -r[0])
    print(f"# stage 2: the best {TOP} cells at 512 episodes", flush=True)
    best = []
    for m, c, _, _ in res[:TOP]:
        m5, ln5, se5 = score(c, 512)
        best.append((m5, c, ln5, se5))
        print(f"TOP {c[0]:5.2f} {c[1]:5.2f} {c[2]:6.2f} {c[3]:6.2f} {c[4]:5.2f} {c[5]:2d} {m5:8.0f} ({se5:4.0f}) {ln5:6.0f}"
              f"   screen {m:.0f}", flush=True)
    print("# surface: best screened return per knob value (the other knobs maximised over)", flush=True)
    names = ["cart", "pole", "margin", "iscale", "damp", "substeps"]
    for j, nm in enumerate(names):
        vals = sorted({c[j] for _, c, _, _ in res})
        row = "  ".join(f"{v:g}: {max(r[0] for r in res if r[1][j] == v):.0f}" for v in vals)
        print(f"#   {nm:9s} {row}", flush=True)
    b = max(best, key=lambda r: r[0])
    print(f"# best cell {dict(zip(names, b[1]))}: {b[0]:.0f} +- {b[3]:.0f} (512 episodes); threshold {THRESHOLD:.0f}: "
          f"{'reached' if b[0] >= THRESHOLD else 'not reached'}", flush=True)


if __name__ == "__main__":
    main()

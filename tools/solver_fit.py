"""Joint fit of the solver's scene parameters against the pretrained policies, on the GPU.

VERDICT r5 (missing 1): the reference's pretrained roboschool policies
(examples/roboschool-weights/enjoy_TF_*.py, weights in tests/golden/policy_*.npz) score below the
registry thresholds on this physics (Walker2D 170 of 2,500, Hopper 2,057, HalfCheetah 1,300 of 3,000,
Ant 777 of 2,500), and every earlier study toggled one rule at a time.  tools/pendulum_fit.py
searched the contact-free dynamics jointly (the double pendulum's plateau); this searches the
parameters the solver takes at run time, jointly, for the contact robots:

  contact ERP (m_erp: Bullet's multibody contact rows use it; pybullet's setDefaultContactERP(0.9)
  writes m_erp2), joint-limit ERP, PGS sweeps (numSolverIterations) and the
  sub-step count (k sub-steps of 16.5 / k ms per env step: numSubSteps).

Every cell runs the policy's episodes through the HIP kernels (float32 for the screen: the
policies score alike at both precisions, tests/test_policies.py), the best PBG_FIT_TOP cells per
robot are re-scored at float64 with PBG_FIT_FULL episodes.  One line per cell, then per robot the
best return for each value of each knob (the other knobs maximised over).  Needs a GPU; prints a
progress line per cell.

  python tools/solver_fit.py > gpurun_out/solver_fit.txt
"""
import itertools
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd.vec_env import VecEnv  # noqa: E402
import policies  # noqa: E402

ENVS = {"HopperPyBulletEnv-v0": 2500.0, "Walker2DPyBulletEnv-v0": 2500.0, "HalfCheetahPyBulletEnv-v0": 3000.0,
        "AntPyBulletEnv-v0": 2500.0, "HumanoidPyBulletEnv-v0": None}
C_ERP = [0.1, 0.2, 0.4, 0.8, 1.0]
L_ERP = [0.1, 0.2, 0.5, 0.9]
ITERS = [5, 10, 25, 50]
SUBS = [4, 8]
SCREEN = int(os.environ.get("PBG_FIT_SCREEN", "128"))
FULL = int(os.environ.get("PBG_FIT_FULL", "512"))
TOP = int(os.environ.get("PBG_FIT_TOP", "4"))
ONLY = os.environ.get("PBG_FIT_ENVS")


def returns(env_id, n, sim, precision, seed=0):
    pi = policies.Policy(env_id)
    env = VecEnv(env_id, n, device="cuda:0", seed=seed, autoreset=False, precision=precision, sim_params=sim)
    nr = env.info.reset_dofs
    obs = env.reset(init_q=torch.from_numpy(policies.reset_draws(n, nr, seed).astype(np.float32)))
    ret = torch.zeros(n, dtype=torch.float64, device=env.device)
    length = torch.zeros(n, dtype=torch.int64, device=env.device)
    alive = torch.ones(n, dtype=torch.bool, device=env.device)
    for t in range(policies.MAX_STEPS):
        r = env.step(pi.torch_act(obs), want_reward64=True)
        ret += torch.where(alive, env.reward64, torch.zeros_like(env.reward64))
        length += alive
        alive &= r.done == 0
        obs = r.obs
        if t % 50 == 49 and not bool(alive.any()):
            break
    out = ret.cpu().numpy(), length.cpu().numpy()
    env.close()
    return out


def main():
    t0 = time.time()
    envs = [e for e in ENVS if not ONLY or e in ONLY.split(",")]
    for env_id in envs:
        base = VecEnv.default_sim_params(env_id)
        rows = []
        for ce, le, it, k in itertools.product(C_ERP, L_ERP, ITERS, SUBS):
            sim = dict(base)
            sim.update(contact_erp=ce, joint_limit_erp=le, solver_iterations=it, frame_skip=k,
                       timestep=base["timestep"] * base["frame_skip"] / k)
            r, ln = returns(env_id, SCREEN, sim, 32)
            rows.append(((ce, le, it, k), float(r.mean()), float(ln.mean())))
            print(f"{env_id} c_erp {ce} l_erp {le} iters {it} substeps {k}: return {r.mean():8.1f} "
                  f"+- {r.std() / np.sqrt(len(r)):6.1f} length {ln.mean():6.1f}  [{time.time() - t0:.0f}s]", flush=True)
        rows.sort(key=lambda x: -x[1])
        default = next(x for x in rows if x[0] == (base["contact_erp"], base["joint_limit_erp"],
                                                    base["solver_iterations"], base["frame_skip"]))
        print(f"== {env_id}: default cell {default[0]} {default[1]:.1f}; threshold {ENVS[env_id]}", flush=True)
        for knob, vals in (("contact_erp", C_ERP), ("joint_limit_erp", L_ERP), ("iterations", ITERS), ("substeps", SUBS)):
            i = ("contact_erp", "joint_limit_erp", "iterations", "substeps").index(knob)
            best = [max(x[1] for x in rows if x[0][i] == v) for v in vals]
            print(f"   {knob:16s} " + "  ".join(f"{v}: {b:7.1f}" for v, b in zip(vals, best)), flush=True)
        for cell, m, ln in rows[:TOP]:
            ce, le, it, k = cell
            sim = dict(base)
            sim.update(contact_erp=ce, joint_limit_erp=le, solver_iterations=it, frame_skip=k,
                       timestep=base["timestep"] * base["frame_skip"] / k)
            r, lnf = returns(env_id, FULL, sim, 64, seed=1)
            print(f"   top {cell}: screen {m:.1f}; float64 x{FULL}: {r.mean():.1f} +- {r.std() / np.sqrt(len(r)):.1f}, "
                  f"length {lnf.mean():.1f}  [{time.time() - t0:.0f}s]", flush=True)
        r, lnf = returns(env_id, FULL, base, 64, seed=1)
        print(f"   default float64 x{FULL}: {r.mean():.1f} +- {r.std() / np.sqrt(len(r)):.1f}, length {lnf.mean():.1f}",
              flush=True)


if __name__ == "__main__":
    main()

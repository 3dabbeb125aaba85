"""Algorithmic FP32 flops per env-step from the
op-counting instantiation of the oracle's physics (oracle/counted.h, pbg_oracle_count_flops):
for each robot, 256 envs are rolled out 200 steps with Philox U(-1, 1) actions and auto-reset
(the bench workload's state distribution), then the next step of every env is counted.
Writes profiles/flops_per_env_step.json and its copy pybullet-gym_amd/perf/ (read by bench.py
for the flop roofline).
Test infrastructure (imports the oracle).  python tools/count_flops.py"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)
import oracle  # noqa: E402
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd import rng  # noqa: E402

ROBOTS = {"pendulum": "InvertedPendulumPyBulletEnv-v0", "hopper": "HopperPyBulletEnv-v0",
          "halfcheetah": "HalfCheetahPyBulletEnv-v0", "ant": "AntPyBulletEnv-v0",
          "humanoid": "HumanoidPyBulletEnv-v0", "walker2d": "Walker2DPyBulletEnv-v0"}


def count(env_id, n=256, warm=200, seed=0x5EED):
    e = oracle.OracleEnvs(env_id, n, nthreads=8, seed=seed)
    ids = np.arange(n)
    epi = np.zeros(n, np.int64)
    obs = e.reset(rng.reset_noise(seed, ids, 0, e.info.NR).astype(np.float64))
    acts = rng.sample_actions(e.info.NA, ids, np.arange(warm + 1), seed=seed)
    for t in range(warm):
        obs, _, done, _ = e.step(acts[t])
        fin = done | (e.aux[:, 2] >= 1000)
        if fin.any():
            epi[fin] += 1
            q = np.zeros((n, e.info.NR))
            for k in np.flatnonzero(fin):
                q[k] = rng.reset_noise(seed, [k], int(epi[k]), e.info.NR)[0]
            e.reset(q, mask=fin, obs=obs)
    L = oracle.lib()
    L.pbg_oracle_count_flops.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    out = np.zeros(7, np.uint64)
    a = np.ascontiguousarray(acts[warm])
    st = np.ascontiguousarray(e.state.copy())
    assert L.pbg_oracle_count_flops(e.rid, n, st.ctypes.data, a.ctypes.data, out.ctypes.data) == 0
    add, mul, div, sq, trans, add_nz, mul_nz = (float(x) / n for x in out)
    return {"flops_per_env_step": add_nz + mul_nz + div + sq + trans,
            "dense_flops_per_env_step": add + mul + div + sq + trans,
            "adds": add_nz, "muls": mul_nz, "divs": div, "sqrts": sq, "sincos": trans,
            "sample": f"{n} envs after {warm} Philox-action steps with auto-reset, one step counted"}


if __name__ == "__main__":
    res = {k: count(v) for k, v in ROBOTS.items()}
    res["_definition"] = ("physics of one env step (apply_action + sub-steps) in FP32 from oracle/pbg_physics.h "
                          "on oracle/counted.h: +,-,*,/,sqrt,sin,cos one flop each; flops_per_env_step skips adds "
                          "and muls with an exactly-zero operand (the dense restatement's structural zeros); the "
                          "float64 observation/reward pack is not counted")
    for path in (os.path.join(REPO, "profiles", "flops_per_env_step.json"),
                 os.path.join(REPO, "pybullet-gym_amd", "perf", "flops_per_env_step.json")):
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
    for k, v in res.items():
        if not k.startswith("_"):
            print(f"{k:12s} {v['flops_per_env_step']:12.0f} flops/env-step (dense {v['dense_flops_per_env_step']:.0f})")

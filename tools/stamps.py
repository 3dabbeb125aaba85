"""Per-phase wave-cycle shares of the step kernel (diagnostic -DPBG_STAMPS build)."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch
import pybulletgym_amd
from pybulletgym_amd import _native
_native.LIB_PATH = os.path.join(REPO, "pybullet-gym_amd", "libpbg_amd_stamps.so")
from pybulletgym_amd.vec_env import VecEnv
L = _native.lib()
L.pbg_debug_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p]
names = ["kin+vel", "composites+M", "cholesky+solve", "limit rows", "contact rows", "PGS (rest)", "integrate", "act+load", "pack",
         "store", "-", "PGS limit rows", "PGS normals", "PGS frictions"]
gang_names = {0: "dist: forward levels", 1: "dist: inertia + motion", 2: "dist: composites", 3: "dist: M + bias",
              10: "factorisation + solves (front-parallel)", 4: "detect",
              11: "rows (jobs)", 5: "PGS", 6: "integrate", 7: "act+load", 13: "pack: bookkeeping loads",
              14: "pack: gather FK", 15: "pack: gather quat", 12: "pack: gather vel, parts, joints",
              8: "pack: walker pack (float64)", 9: "store (+ auto-reset)"}
AUTORESET = os.environ.get("PBG_STAMPS_AUTORESET", "1") != "0"
# ENV:N[:GANG_DIST[:GANG_LANES[:PRECISION]]]  (GANG_DIST 0/1 forces the gang kernel's replicated /
# distributed dynamics, -1 the plan's; GANG_LANES 16 / 32 the gang width, -1 the plan's; PRECISION 64:
# the float64 handle)
for spec in (sys.argv[1:] or ["AntPyBulletEnv-v0:16384"]):
    env_id, n, *rest = spec.split(":")
    n = int(n)
    env = VecEnv(env_id, n, seed=1, autoreset=AUTORESET, gang_dist=int(rest[0]) if rest else -1,
                 gang_lanes=int(rest[1]) if len(rest) > 1 else -1, precision=int(rest[2]) if len(rest) > 2 else 32)
    env.reset()
    acts = torch.rand((30, n, env.info.action_dim), device="cuda") * 2 - 1
    for i in range(200): env.step(acts[i % 30])  # pre-roll off the reset pose, as bench.py
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    rid = _native.ROBOT_IDS[env_id]
    assert L.pbg_debug_stamps(rid, buf) == 0, env_id
    steps = 20
    for i in range(steps): env.step(acts[10 + i])
    torch.cuda.synchronize()
    assert L.pbg_debug_stamps(rid, buf) == 0, env_id
    lpe = max(1, env.info.lanes_per_env)
    if lpe == 1:  # lane kernel: workgroups of 16/32/64 lanes, one wave each (plan_* in pbg_robot.hip)
        per_cu, b = -(-n // 256), 16
        while b < per_cu and b < 64: b *= 2
        waves = -(-n // b)
    else:
        waves = -(-n * lpe // 64)
    tot = sum(buf[i] for i in range(16))
    print(f"{env_id} n={n} lanes/env={lpe}: cycles per wave per env-step = {tot / waves / steps:.0f}")
    labels = gang_names if lpe >= 16 else dict(enumerate(names))
    for i in sorted(labels, key=lambda k: list(labels).index(k)):
        print(f"   {labels[i]:26s} {buf[i] / waves / steps:10.0f}  {100.0 * buf[i] / tot:5.1f}%")

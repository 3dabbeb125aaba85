"""Gang contact-record bound checks (dev tool): steps the gang robots with the diagnostic
-DPBG_DEV_CHECKS library (`make -C pybullet-gym_amd checks`), whose contact_at() asserts that
every contact record lies inside its env's LDS region or workspace slice, at the parity tests'
env count and at the bench's, with the plan's LDS capacity and with every contact in the
workspace (lds_rows = 0).  A failed device assert aborts the process."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd import _native  # noqa: E402

_native.LIB_PATH = os.path.join(REPO, "pybullet-gym_amd", "libpbg_amd_checks.so")
from pybulletgym_amd.vec_env import VecEnv, sample_actions  # noqa: E402

ENVS = ["HumanoidPyBulletEnv-v0", "HumanoidFlagrunPyBulletEnv-v0", "HumanoidFlagrunHarderPyBulletEnv-v0",
        "AtlasPyBulletEnv-v0", "Walker2DPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0", "HopperPyBulletEnv-v0"]
for env_id in ENVS:
    for n in (256, 4096):
        for lds_rows in (-1, 0):
            env = VecEnv(env_id, n, seed=7, autoreset=True, lds_rows=lds_rows, precision=32)
            env.reset()
            acts = sample_actions(env.info.action_dim, n, 60, seed=7)
            for i in range(60):
                env.step(acts[i])
            torch.cuda.synchronize()
            print(f"{env_id:38s} n={n:5d} lds_rows={lds_rows:2d} ok (cap {env.info.lds_rows})", flush=True)
            env.close()
print("bounds ok")

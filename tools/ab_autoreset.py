"""Step time with and without auto-reset (dev tool): how much the reset path costs."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch
import pybulletgym_amd
from pybulletgym_amd.vec_env import VecEnv
for env_id, n in [("HumanoidPyBulletEnv-v0", 4096), ("AntPyBulletEnv-v0", 16384)]:
    for ar in (True, False):
        env = VecEnv(env_id, n, seed=2, autoreset=ar, precision=32)
        env.reset()
        K = 100
        acts = torch.rand((K, n, env.info.action_dim), device="cuda") * 2 - 1
        for i in range(10): env.step(acts[i])
        torch.cuda.synchronize(); t = time.time()
        dn = 0
        for i in range(K):
            r = env.step(acts[i])
            if i % 10 == 0:
                dn += int(r.done.sum())
        torch.cuda.synchronize(); dt = time.time() - t
        print(f"{env_id:28s} autoreset={ar!s:5s} {dt / K * 1e3:8.3f} ms/step  done/step~{dn / 10:.0f}", flush=True)
        env.close()

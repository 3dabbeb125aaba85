"""Throughput of the step kernel per robot at the BASELINE config sizes (dev tool)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch
import pybulletgym_amd
from pybulletgym_amd.vec_env import VecEnv
cfg = [("InvertedPendulumPyBulletEnv-v0", 16384), ("HopperPyBulletEnv-v0", 4096), ("HalfCheetahPyBulletEnv-v0", 8192),
       ("AntPyBulletEnv-v0", 16384), ("HumanoidPyBulletEnv-v0", 4096), ("Walker2DPyBulletEnv-v0", 4096),
       ("InvertedPendulumSwingupPyBulletEnv-v0", 16384), ("InvertedDoublePendulumPyBulletEnv-v0", 16384),
       ("HumanoidFlagrunPyBulletEnv-v0", 4096), ("HopperMuJoCoEnv-v0", 4096), ("Walker2DMuJoCoEnv-v0", 4096),
       ("HalfCheetahMuJoCoEnv-v0", 8192), ("AntMuJoCoEnv-v0", 16384), ("HumanoidMuJoCoEnv-v0", 4096)]
if len(sys.argv) > 1:
    cfg = [(a, int(b)) for a, b in (x.split(":") for x in sys.argv[1:])]
for env_id, n in cfg:
    env = VecEnv(env_id, n, seed=2, autoreset=True, precision=32)
    env.reset()
    K = 100
    acts = torch.rand((K, n, env.info.action_dim), device="cuda") * 2 - 1
    for i in range(10): env.step(acts[i])
    torch.cuda.synchronize(); t = time.time()
    for i in range(K): env.step(acts[i])
    torch.cuda.synchronize(); dt = time.time() - t
    print(f"{env_id:32s} n={n:6d}  {dt / K * 1e3:8.3f} ms/step  {n * K / dt:10.3g} env-steps/s", flush=True)

"""Step time against the gang kernel's LDS contact capacity (dev tool: how much the rows swept from
the device workspace cost).  python tools/cap_probe.py ENV:N CAP [CAP ...]  (CAP -1: the plan's own)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pybulletgym_amd  # noqa: F401
from pybulletgym_amd.vec_env import VecEnv, sample_actions
env_id, n = sys.argv[1].split(":")
n = int(n)
for cap in [int(c) for c in sys.argv[2:]]:
    env = VecEnv(env_id, n, seed=0x5EED, autoreset=True, lds_rows=cap, precision=32)
    env.reset()
    K, P = 300, 200
    acts = sample_actions(env.info.action_dim, n, P + K, seed=0x5EED)
    for i in range(P): env.step(acts[i])
    g = env.capture([acts[P + i] for i in range(K)])
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / K)
    print(f"{env_id} n={n} cap={cap} (in force {env.info.lds_rows}) {min(ts):.4f} ms", flush=True)
    del g, env

"""Float64 quad vs float32 quad vs float64 lane, one step from the same state (dev diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pybulletgym_amd  # noqa
from pybulletgym_amd.vec_env import VecEnv


def rel(a, b):
    return (np.abs(a - b) / np.maximum(1.0, np.abs(b))).max(axis=0)


for n in (16, 64):
    for init in (False, True):
        q64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64)
        q32 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=32)
        l64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64, kernel=0)
        r = np.random.default_rng(7)
        if init:
            q64.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, 8)).astype(np.float32)))
        else:
            q64.reset()
        phys, aux = q64.get_state()
        q32.set_state(phys, aux)
        l64.set_state(phys, aux)
        a = torch.zeros((n, 8), device="cuda")
        for e in (q64, q32, l64):
            e.step(a)
        s64, s32, sl = (e.get_state()[0].cpu().numpy() for e in (q64, q32, l64))
        print(f"n={n} init_q={init}")
        print("  q64 vs l64:", np.array2string(rel(s64, sl), precision=1, max_line_width=250))
        print("  q32 vs l64:", np.array2string(rel(s32, sl), precision=1, max_line_width=250))
        print("  q64 vs q32 per env:", np.array2string((np.abs(s64 - s32) / np.maximum(1, np.abs(s32))).max(axis=1), precision=1, max_line_width=250))

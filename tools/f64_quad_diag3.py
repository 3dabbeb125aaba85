"""Float64 quad vs float64 lane under scene variants (dev diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pybulletgym_amd  # noqa
from pybulletgym_amd.vec_env import VecEnv

n = 64
for sim in ({"frame_skip": 1}, {"frame_skip": 2}, {"frame_skip": 4}, {"frame_skip": 1, "solver_iterations": 1},
            {"frame_skip": 1, "gravity": 0.0}):
    sp = VecEnv.default_sim_params("AntPyBulletEnv-v0")
    sp.update(sim)
    q64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64, sim_params=sp)
    l64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64, kernel=0, sim_params=sp)
    q64.reset()
    phys, aux = q64.get_state()
    l64.set_state(phys, aux)
    a = torch.zeros((n, 8), device="cuda")
    q64.step(a)
    l64.step(a)
    s64, sl = (e.get_state()[0].cpu().numpy() for e in (q64, l64))
    r = (np.abs(s64 - sl) / np.maximum(1.0, np.abs(sl)))
    print(sim, "max per word:", np.array2string(r.max(axis=0), precision=1, max_line_width=250))
    print("   per env:", np.array2string(r.max(axis=1)[:16], precision=1, max_line_width=250))
    print("   env0 q64:", np.array2string(s64[0], precision=4, max_line_width=250))
    print("   env0 l64:", np.array2string(sl[0], precision=4, max_line_width=250))

"""Float64 quad vs float64 lane, frame_skip 1, several batch shapes; optional debug library
(dev diagnostic).  usage: f64_quad_diag4.py [libname]"""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pybulletgym_amd  # noqa
from pybulletgym_amd import _native
if len(sys.argv) > 1:
    _native.LIB_PATH = os.path.join(os.path.dirname(_native.__file__), sys.argv[1])
from pybulletgym_amd.vec_env import VecEnv

sp = VecEnv.default_sim_params("AntPyBulletEnv-v0")
sp.update({"frame_skip": 1})
for n, off in ((1, 0), (4, 0), (16, 0), (16, 2), (64, 0)):
    q64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, env_offset=off, autoreset=False, precision=64, sim_params=sp)
    l64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, env_offset=off, autoreset=False, precision=64, kernel=0, sim_params=sp)
    q64.reset()
    phys, aux = q64.get_state()
    l64.set_state(phys, aux)
    a = torch.zeros((n, 8), device="cuda")
    q64.step(a, want_contacts=True)
    l64.step(a, want_contacts=True)
    s64, sl = (e.get_state()[0].cpu().numpy() for e in (q64, l64))
    r = (np.abs(s64 - sl) / np.maximum(1.0, np.abs(sl))).max(axis=1)
    print(f"n={n} off={off} bad envs (global):", [off + i for i in np.nonzero(r > 1e-9)[0]],
          "nc:", l64.ncontact.cpu().numpy()[:16].tolist(), flush=True)

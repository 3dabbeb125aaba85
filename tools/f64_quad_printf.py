"""One step of the float32 and the float64 quad kernels from the same state, with the debug
library's per-phase printf (libpbg_amd_tdbg.so, -DPBG_TEAM_DEBUG; dev diagnostic)."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pybulletgym_amd  # noqa
from pybulletgym_amd import _native
_native.LIB_PATH = os.path.join(os.path.dirname(_native.__file__), "libpbg_amd_tdbg.so")
from pybulletgym_amd.vec_env import VecEnv

n = 16
e64 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64)
e32 = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=32)
e64.reset()
phys, aux = e64.get_state()
e32.set_state(phys, aux)
torch.cuda.synchronize()
a = torch.zeros((n, 8), device="cuda")
print("=== f32", flush=True)
e32.step(a)
torch.cuda.synchronize()
print("=== f64", flush=True)
e64.step(a)
torch.cuda.synchronize()
print("=== done", flush=True)

"""Bitwise A/B of two builds of libpbg_amd.so (dev tool): each build rolls the same envs with the
same Philox actions in its own subprocess; the state records after every step must agree bit for
bit (a refactor that claims to keep the arithmetic), or the report gives the largest difference.
python tools/ab_bits.py LIB_A LIB_B ENV:N:STEPS[:GANG_LANES[:PRECISION[:LDS_ROWS]]] ..."""
import os
import subprocess
import sys
import tempfile

import numpy as np

CHILD = r'''
import sys, torch, numpy as np
sys.path.insert(0, "{repo}")
import pybulletgym_amd
from pybulletgym_amd import _native
_native.LIB_PATH = "{lib}"
from pybulletgym_amd.vec_env import VecEnv, sample_actions
env = VecEnv("{env}", {n}, seed=0x5EED, autoreset=True, gang_lanes={gl}, precision={pr}, lds_rows={lr})
env.reset()
acts = sample_actions(env.info.action_dim, {n}, {steps}, seed=0x5EED)
out = []
for i in range({steps}):
    env.step(acts[i])
    phys, aux = env.get_state()
    out.append(phys.cpu().numpy())
np.save("{out}", np.stack(out))
print(env.info.lanes_per_env if hasattr(env.info, "lanes_per_env") else "")
'''


def run(lib, out, env, n, steps, gl, pr, lr):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = CHILD.format(repo=repo, lib=os.path.abspath(lib), env=env, n=n, steps=steps, gl=gl, pr=pr, lr=lr, out=out)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    if r.returncode:
        raise RuntimeError(r.stderr[-2000:])
    return np.load(out)


if __name__ == "__main__":
    a, b = sys.argv[1], sys.argv[2]
    with tempfile.TemporaryDirectory() as td:
        for spec in sys.argv[3:]:
            env, n, steps, *opt = spec.split(":")
            gl = int(opt[0]) if opt else -1
            pr = int(opt[1]) if len(opt) > 1 else 32
            lr = int(opt[2]) if len(opt) > 2 else -1
            A = run(a, os.path.join(td, "a.npy"), env, int(n), int(steps), gl, pr, lr)
            B = run(b, os.path.join(td, "b.npy"), env, int(n), int(steps), gl, pr, lr)
            same = np.array_equal(A.view(np.uint64), B.view(np.uint64))
            first = next((t for t in range(A.shape[0]) if not np.array_equal(A[t].view(np.uint64), B[t].view(np.uint64))), None)
            d = np.abs(A - B)
            print(f"{spec}: {'BITWISE EQUAL' if same else 'DIFFER'} first differing step {first} "
                  f"max |diff| {np.nanmax(d):.3e} envs differing at the end {(d[-1].max(axis=1) > 0).sum()}/{n}", flush=True)

"""A/B timing of two builds of libpbg_amd.so on the same GPU (dev tool): each variant runs in
its own subprocess (the library is loaded once per process), alternating A, B, A, B; each run
is bench-like (Philox actions, pre-roll, one HIP graph of the timed steps).
python tools/ab_lib.py LIB_A LIB_B ENV:N[:GANG_DIST[:GANG_LANES]] ...
LIB_A / LIB_B: a libpbg_amd.so (run with this tree's Python package) or a directory holding a
whole tree snapshot (its pybulletgym_amd.py, pybullet-gym_amd/ and built library), for a base
whose C-ABI predates the current package's.  (The snapshots live under ab/, which .gpurunignore
keeps off the GPU box between A/B campaigns: drop that line to upload them.)"""
import os
import subprocess
import sys

CHILD = r'''
import sys, time, torch
sys.path.insert(0, "{repo}")
import pybulletgym_amd
from pybulletgym_amd import _native
_native.LIB_PATH = "{lib}"
from pybulletgym_amd.vec_env import VecEnv, sample_actions
env_id, n = "{env}", {n}
kw = dict(gang_dist={gd})
if {gl} > 0: kw["gang_lanes"] = {gl}
kw["precision"] = {pr}
env = VecEnv(env_id, n, seed=0x5EED, autoreset=True, **kw)
env.reset()
K, P = 300, 200
acts = sample_actions(env.info.action_dim, n, P + K, seed=0x5EED)
for i in range(P): env.step(acts[i])
g = env.capture([acts[P + i] for i in range(K)])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
print("%.5f" % (e0.elapsed_time(e1) / K))
'''


def run(lib, env, n, gd=-1, gl=-1, pr=32):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if os.path.isdir(lib):
        repo, lib = lib, os.path.join(lib, "pybullet-gym_amd", "libpbg_amd.so")
    code = CHILD.format(repo=os.path.abspath(repo), lib=os.path.abspath(lib), env=env, n=n, gd=gd, gl=gl, pr=pr)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if out.returncode:
        raise RuntimeError(out.stderr[-2000:])
    return float(out.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    a, b = sys.argv[1], sys.argv[2]
    for spec in sys.argv[3:]:
        env, n, *opt = spec.split(":")  # ENV:N[:GANG_DIST[:GANG_LANES[:PRECISION]]]
        gd = int(opt[0]) if opt else -1
        gl = int(opt[1]) if len(opt) > 1 else -1
        pr = int(opt[2]) if len(opt) > 2 else 32
        ta, tb = [], []
        for _ in range(2):
            ta.append(run(a, env, int(n), gd, gl, pr))
            tb.append(run(b, env, int(n), gd, gl, pr))
        print(f"{env:28s} n={n:>6s} f{pr} A {min(ta):.4f} ms  B {min(tb):.4f} ms  B/A {min(tb) / min(ta):.3f}", flush=True)

"""A/B of plan variants of ONE build in one process (dev tool): each variant is a VecEnv option set;
the variants' timed windows alternate (R rounds x K steps, CUDA events around the window), the
median per variant is printed.  Also checks the variants step the same states to within TOL.

  python tools/ab_variant.py ENV_ID N PRECISION 'gang_dist=1' 'gang_dist=0' [--rounds 7 --steps 200]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd.vec_env import VecEnv, sample_actions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("env_id")
    ap.add_argument("n", type=int)
    ap.add_argument("precision", type=int)
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--lib", default=None, help="a diagnostic build instead of the product library")
    a = ap.parse_args()
    if a.lib:
        from pybulletgym_amd import _native
        _native.LIB_PATH = os.path.abspath(a.lib)
    envs = []
    for v in a.variants:
        kw = {k: int(x) for k, x in (p.split("=") for p in v.split(",") if p)}
        e = VecEnv(a.env_id, a.n, seed=5, autoreset=True, precision=a.precision, **kw)
        e.reset()
        envs.append(e)
        i = e.info
        print(f"{v or 'default'}: lanes/env {i.lanes_per_env}, block {i.block}, LDS {i.lds_bytes} B, lds_rows "
              f"{i.lds_rows}, VGPR+AGPR {i.vgprs}, scratch {i.scratch_bytes} B", flush=True)
    acts = sample_actions(envs[0].info.action_dim, a.n, a.steps, seed=11)
    # same-state check: every variant from variant 0's state after 50 steps, 20 steps
    for t in range(50):
        envs[0].step(acts[t])
    phys, aux = envs[0].get_state()
    outs = []
    for e in envs:
        e.set_state(phys, aux)
        for t in range(20):
            e.step(acts[t])
        outs.append(e.get_state()[0].cpu().numpy())
    for v, o in zip(a.variants[1:], outs[1:]):
        rel = np.abs(o - outs[0]) / np.maximum(1.0, np.abs(outs[0]))
        print(f"{v}: 20 steps from the same state, max rel state diff vs {a.variants[0]} {np.nanmax(rel):.3g}", flush=True)
    times = [[] for _ in envs]
    for r in range(a.rounds):
        for i, e in enumerate(envs):
            for t in range(10):
                e.step(acts[t])
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s0.record()
            for t in range(a.steps):
                e.step(acts[t])
            s1.record()
            torch.cuda.synchronize()
            times[i].append(s0.elapsed_time(s1) / a.steps)
    for v, ts in zip(a.variants, times):
        print(f"{a.env_id} n={a.n} f{a.precision} {v or 'default'}: median {np.median(ts):.4f} ms/step "
              f"(min {min(ts):.4f}, max {max(ts):.4f})", flush=True)


if __name__ == "__main__":
    main()

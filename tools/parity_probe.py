"""Diagnostic (GPU box): replay dumped class-A outlier env-steps (tools/parity_dump.py) on the
GPU from their exact states, unperturbed and under tiny state perturbations, for each kernel
variant; writes gpurun_out/<tag>/probe.npz.  python tools/parity_probe.py ENV DUMP_TAG TAG"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd.vec_env import VecEnv  # noqa: E402


def main(env_id, dump_tag, tag):
    z = np.load(os.path.join(HERE, "_dumps", dump_tag + ".npz"))
    st, ax, act = z["state"], z["aux"], z["act"]
    n = len(st)
    rng = np.random.default_rng(0)
    out = {}
    for kernel in (-1, 0, 2):
        res = []
        for rep in range(6):
            s = st.copy()
            if rep > 0:  # relative perturbation ~1e-6 of every state word
                s = s * (1.0 + rng.uniform(-1e-6, 1e-6, s.shape))
            env = VecEnv(env_id, n, seed=7, autoreset=False, kernel=kernel, precision=32)
            env.set_state(torch.from_numpy(s), torch.from_numpy(ax))
            r = env.step(torch.from_numpy(act).float().cuda())
            res.append(r.obs.cpu().numpy().copy())
            env.close()
        out[f"k{kernel}"] = np.stack(res)
    os.makedirs(os.path.join("gpurun_out", tag), exist_ok=True)
    np.savez(os.path.join("gpurun_out", tag, "probe.npz"), **out)
    print("ok", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(*sys.argv[1:4])

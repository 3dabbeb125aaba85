"""Diagnostic (GPU box): teacher-forced steps of one env id; dumps the class-A env-steps
(same contact set, float32 oracle within 2e-5 of float64) whose GPU obs error exceeds 1e-4:
input state/aux records, action, GPU / float64 / float32 obs, to gpurun_out/<tag>/worst.npz.
python tools/parity_dump.py ENV N STEPS TAG"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import oracle  # noqa: E402
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd.vec_env import VecEnv, sample_actions  # noqa: E402


def rel(a, b):
    return np.abs(a.astype(np.float64) - b) / np.maximum(1.0, np.abs(b))


def main(env_id, n, steps, tag, kernel=-1):
    env = VecEnv(env_id, n, seed=7, autoreset=True, kernel=kernel, precision=32)
    env.reset()
    orc = oracle.OracleEnvs(env_id, n, nthreads=16, seed=7)
    prb = oracle.OracleEnvs(env_id, n, nthreads=16, seed=7, precision=32)
    acts = sample_actions(env.info.action_dim, n, steps, seed=7)
    keep = {k: [] for k in ("state", "aux", "act", "og", "oo", "op", "err", "step")}
    for t in range(steps):
        phys, aux = env.get_state()
        st, ax = phys.cpu().numpy(), aux.cpu().numpy()
        orc.state[:] = st; orc.aux[:] = ax
        prb.state[:] = st; prb.aux[:] = ax
        res = env.step(acts[t], want_contacts=True)
        done = res.done.bool()
        og = torch.where(done[:, None], res.terminal_obs, res.obs).cpu().numpy()
        sg = env.contact_sig.cpu().numpy().view(np.uint32)
        a = acts[t].cpu().numpy()
        oo, _, _, _ = orc.step(a)
        op, _, _, _ = prb.step(a)
        probe = rel(op, oo).max(1)
        e = rel(og, oo)
        bad = (sg == orc.csig) & (prb.csig == orc.csig) & (probe <= 2e-5) & (e.max(1) > 1e-4)
        for i in np.flatnonzero(bad):
            for k, v in (("state", st[i]), ("aux", ax[i]), ("act", a[i]), ("og", og[i]), ("oo", oo[i]), ("op", op[i]),
                         ("err", e[i]), ("step", t)):
                keep[k].append(v)
    out = os.path.join("gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    np.savez(os.path.join(out, "worst.npz"), **{k: np.array(v) for k, v in keep.items()})
    print(env_id, "bad class-A env-steps:", len(keep["step"]), "of", n * steps)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else -1)

"""Float64 lane kernel of the Humanoid with the physics' own sin / cos (the round-6 "second instance",
DESIGN.md section 4; dev tool).  Teacher-forced from the 32-lane gang kernel's states: each step the
lane kernel runs twice from the same state, after every SIMD's register file is set to two different
patterns (tools/libvgpr_poison.so), and both results are compared bitwise and against the gang step.

  python tools/lane_owntrig_probe.py LIB [ENV_ID] [N] [STEPS]
  python tools/lane_owntrig_probe.py LIB --bisect [ENV_ID] [N]   # which registers: subsets set to a NaN
      high word, the rest 1.0's, halved while the lane step differs from the all-1.0 run
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd import _native  # noqa: E402


def bisect(lib, env_id, n):
    _native.LIB_PATH = lib
    from pybulletgym_amd.vec_env import VecEnv, sample_actions
    VL = ctypes.CDLL(os.path.join(HERE, "libvgpr_poison.so"))
    VL.vgpr_poison_mask.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    g = VecEnv(env_id, n, seed=3, autoreset=False, precision=64)
    ln = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, kernel=0)
    g.reset()
    acts = sample_actions(g.info.action_dim, n, 12, seed=21)
    for t in range(10):
        g.step(acts[t])
    phys, aux = g.get_state()
    cnt = [0]

    def trial(nan_regs):
        m = np.zeros(16, np.uint32)
        for r in nan_regs:
            m[r >> 5] |= np.uint32(1) << np.uint32(r & 31)
        ln.set_state(phys, aux)
        torch.cuda.synchronize()
        assert VL.vgpr_poison_mask(0x7FF80000, 0x3FF00000, m.ctypes.data, 8192) == 0
        ln.step(acts[10])
        cnt[0] += 1
        return ln.get_state()[0].cpu().numpy()

    ref = trial([])
    print(f"all-1.0 twice identical: {(trial([]).view(np.uint64) == ref.view(np.uint64)).all()}; all-NaN differs: "
          f"{(trial(range(512)).view(np.uint64) != ref.view(np.uint64)).any()}", flush=True)
    found = []

    def rec(regs):
        if cnt[0] >= 400:
            return
        z = trial(regs)
        d = int((z.view(np.uint64) != ref.view(np.uint64)).any(axis=1).sum())
        if d == 0:
            return
        if len(regs) == 1:
            found.append((regs[0], d))
            return
        h = len(regs) // 2
        rec(regs[:h])
        rec(regs[h:])

    rec(list(range(512)))
    print(f"{env_id} float64 lane kernel: registers whose contents change the step ({cnt[0]} trials): " +
          ", ".join(f"{'v' if r < 256 else 'a'}{r % 256} ({d} envs)" for r, d in found), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "--bisect":
        bisect(os.path.abspath(sys.argv[1]), sys.argv[3] if len(sys.argv) > 3 else "HumanoidPyBulletEnv-v0",
               int(sys.argv[4]) if len(sys.argv) > 4 else 256)
        return
    lib = os.path.abspath(sys.argv[1])
    env_id = sys.argv[2] if len(sys.argv) > 2 else "HumanoidPyBulletEnv-v0"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    _native.LIB_PATH = lib
    from pybulletgym_amd.vec_env import VecEnv, sample_actions
    VL = ctypes.CDLL(os.path.join(HERE, "libvgpr_poison.so"))
    VL.vgpr_poison.argtypes = [ctypes.c_uint32, ctypes.c_int]
    g = VecEnv(env_id, n, seed=3, autoreset=False, precision=64)
    ln = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, kernel=0)
    print(f"{os.path.basename(lib)} {env_id}: gang lanes/env {g.info.lanes_per_env}, lane kernel scratch "
          f"{ln.info.scratch_bytes} B, VGPR+AGPR {ln.info.vgprs}", flush=True)
    g.reset()
    acts = sample_actions(g.info.action_dim, n, steps, seed=21)
    diff_ab = bad_a = bad_b = same_n = 0
    worst = 0.0
    for t in range(steps):
        phys, aux = g.get_state()
        outs = []
        for base in (0x7FF80000, 0x3FF00000):
            ln.set_state(phys, aux)
            torch.cuda.synchronize()
            assert VL.vgpr_poison(base, 8192) == 0
            ln.step(acts[t], want_contacts=True)
            outs.append((ln.get_state()[0].cpu().numpy(), ln.contact_sig.cpu().numpy().copy()))
        g.step(acts[t], want_contacts=True)
        sg, cg = g.get_state()[0].cpu().numpy(), g.contact_sig.cpu().numpy()
        (sa, ca), (sb, cb) = outs
        diff_ab += int((sa.view(np.uint64) != sb.view(np.uint64)).any(axis=1).sum())
        same = ca == cg
        same_n += int(same.sum())
        for s_, name in ((sa, "a"), (sb, "b")):
            rel = (np.abs(s_ - sg) / np.maximum(1.0, np.abs(sg))).max(axis=1)
            k = int((~(rel[same] <= 1e-9)).sum())
            worst = max(worst, float(np.nanmax(rel[same])) if same.any() else 0.0)
            if name == "a":
                bad_a += k
            else:
                bad_b += k
    print(f"{steps} steps x {n} envs: env-steps whose lane state differs between the two register patterns "
          f"{diff_ab}; same-contact-set env-steps {same_n}, above 1e-9 vs the gang kernel: {bad_a} (NaN-pattern "
          f"registers) / {bad_b} (1.0-pattern registers), worst {worst:.3g}", flush=True)


if __name__ == "__main__":
    main()

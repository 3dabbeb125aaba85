"""Float64 quad-kernel diagnostic (replaces the round-5 f64_quad_diag*/printf scripts).

`make -C pybullet-gym_amd trace` builds two diagnostic libraries that differ only in the machine
schedule of team_step_kernel<F64<Ant>,16> (csrc/pbg_robot.hip -DPBG_TEAM64_TU -DPBG_TRACE64):
libpbg_trace_def.so (the default scheduler) and libpbg_trace_trk.so (the AMDGPU register-pressure
trackers, the product's flag).  Both record the per-lane values of the quad kernel's phases
(pbg_team.hip TRACE64: composites, detection, mass matrix, factorisation, solves, limit rows, PGS,
integration) in the last sub-step.  For each library, in its own process:

  64 Ant envs, float64, one env step of ONE sub-step (frame_skip 1), from the same reset state,
  zero and then random actions; the quad kernel's state against the float64 lane kernel (kernel=0,
  the product's default-schedule lane TU) from the same input state; and the trace.

  python tools/f64_quad_trace.py [LIB ...]          # default: both trace libraries
  python tools/f64_quad_trace.py --child LIB OUT.npz

Prints per library the envs whose state differs from the lane kernel by > 1e-9, and per phase the
first trace slot where the two schedules differ (relative 1e-12) or turn non-finite.
"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PH = ["composites", "detection", "mass matrix", "factorisation", "solves", "limit rows", "PGS", "integration"]
SLOTS = [["tm", "tp1.x", "tF.x", "tF.z", "tN.y", "tJ0", "tJ5", "kb"],
         ["n0", "nc", "ci", "act", "base_bits", "sdist0", "sP0.x", "sP0.z"],
         ["Lbr00", "Lbr10", "Lbr11", "Lgb00", "Lgb51", "Mbb33", "rb0", "rB2"],
         ["Ld0", "Ld1", "Lbb00", "Lbb55", "Ldb5", "Lbb53", "Lgb20", "Lbr10"],
         ["yb0", "yB0", "xB2", "xb0", "nB2", "nb0", "ub0", "uB5"],
         ["Om0", "Orm0", "Otl0", "Oth0", "BY000", "BY101", "Byb000", "Om_last"],
         ["uBs0", "uBs1", "ub0", "ub_last", "uB0", "uB5", "nc", "uB2"],
         ["nB0", "nB3", "nb0", "nb_last", "qd0", "bv2", "bw0", "bq3"]]


def child(lib, out):
    import ctypes
    import torch
    sys.path.insert(0, REPO)
    import pybulletgym_amd  # noqa: F401
    from pybulletgym_amd import _native
    _native.LIB_PATH = lib
    from pybulletgym_amd.vec_env import VecEnv
    L = _native.lib()
    traced = hasattr(L, "pbg_debug_trace64")  # libpbg_trace_plain.so: the default schedule without the trace
    if traced:
        L.pbg_debug_trace64.argtypes = [ctypes.c_void_p]
    n = 64
    sim = {"frame_skip": 1}
    q = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64, sim_params=sim)
    ln = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False, precision=64, sim_params=sim, kernel=0)
    assert q.info.lanes_per_env == 4 and ln.info.lanes_per_env == 1
    r = np.random.default_rng(7)
    q.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, q.info.reset_dofs)).astype(np.float32)))
    res = {}
    # PBG_POISON=0xPATTERN: every CU's LDS filled with the pattern before the quad step (pbg_debug_poison
    # of PBG_POISON_LIB, default the product library -- so a library without the entry point, such as
    # round 5's, can be probed for reads of LDS it never wrote)
    # PBG_POISON_RANGE=b:e: only LDS words [b, e) get the pattern, the rest zero (tools/liblds_poison.so;
    # tools/lds_poison_bisect.py)
    poison = os.environ.get("PBG_POISON")
    prange = os.environ.get("PBG_POISON_RANGE")
    if poison and prange:
        RL = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblds_poison.so"))
        RL.lds_poison_range.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        b_, e_ = (int(x) for x in prange.split(":"))
    elif poison:
        PL = ctypes.CDLL(os.environ.get("PBG_POISON_LIB", os.path.join(REPO, "pybullet-gym_amd", "libpbg_amd.so")))
        PL.pbg_debug_poison.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    # PBG_VGPR_POISON=0xBASE: every SIMD's whole register file (256 VGPRs + 256 AGPRs) set to BASE | index
    # right before the quad step (tools/libvgpr_poison.so), after any LDS poison
    # PBG_VGPR_POISON=A:B:W0,..,W15 (hex): register r gets A where bit r of the 512-bit mask is set, else B
    vpoison = os.environ.get("PBG_VGPR_POISON")
    if vpoison:
        VL = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvgpr_poison.so"))
        VL.vgpr_poison.argtypes = [ctypes.c_uint32, ctypes.c_int]
        VL.vgpr_poison_mask.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        if ":" in vpoison:
            pa, pb, pm = vpoison.split(":")
            vmask = np.array([int(x, 16) for x in pm.split(",")], dtype=np.uint32)
            assert vmask.size == 16

    def vgpr_poison():
        if ":" in vpoison:
            assert VL.vgpr_poison_mask(int(pa, 16), int(pb, 16), vmask.ctypes.data, 8192) == 0
        else:
            assert VL.vgpr_poison(int(vpoison, 16), 8192) == 0
    for tag in ("zero", "rand"):
        phys, aux = q.get_state()
        ln.set_state(phys, aux)
        a = torch.zeros((n, 8), device="cuda") if tag == "zero" else \
            torch.from_numpy(r.uniform(-1, 1, (n, 8)).astype(np.float32)).cuda()
        if vpoison and not poison:
            torch.cuda.synchronize()
            vgpr_poison()
            torch.cuda.synchronize()
        if poison:
            torch.cuda.synchronize()
            if prange:
                assert RL.lds_poison_range(int(poison, 16), b_, e_) == 0
            else:
                assert PL.pbg_debug_poison(None, int(poison, 16), None) == 0
            torch.cuda.synchronize()
            if vpoison:
                vgpr_poison()
                torch.cuda.synchronize()
        q.step(a)
        torch.cuda.synchronize()
        buf = np.full(256 * 8 * 8, np.nan)
        if traced:
            assert L.pbg_debug_trace64(buf.ctypes.data) == buf.size
        ln.step(a)
        res[f"{tag}_trace"] = buf.reshape(256, 8, 8)
        res[f"{tag}_quad"] = q.get_state()[0].cpu().numpy()
        res[f"{tag}_lane"] = ln.get_state()[0].cpu().numpy()
        res[f"{tag}_in"] = phys.cpu().numpy()
    np.savez(out, **res)


def main(libs):
    outs = {}
    for lib in libs:
        out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", REPO), "gpurun_out",
                           "f64_trace_" + os.path.basename(lib).replace(".so", "")
                           + (f"_poison{os.environ['PBG_POISON']}" if os.environ.get("PBG_POISON") else "") + ".npz")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.check_call([sys.executable, __file__, "--child", lib, out], timeout=300)
        outs[lib] = np.load(out)
    for lib, z in outs.items():
        for tag in ("zero", "rand"):
            rel = (np.abs(z[f"{tag}_quad"] - z[f"{tag}_lane"]) / np.maximum(1.0, np.abs(z[f"{tag}_lane"]))).max(axis=1)
            bad = np.flatnonzero(~(rel <= 1e-9))
            print(f"{os.path.basename(lib)} {tag}: quad vs lane, {len(bad)} of {len(rel)} envs above 1e-9 "
                  f"(max {np.nanmax(rel):.3g}, non-finite envs {int((~np.isfinite(z[f'{tag}_quad'])).any(axis=1).sum())})")
            if len(bad):  # which state words (base p 0-2 | quat 3-6 | v 7-9 | w 10-12 | q 13.. | qd ..)
                w = (np.abs(z[f"{tag}_quad"] - z[f"{tag}_lane"]) / np.maximum(1.0, np.abs(z[f"{tag}_lane"]))).max(axis=0)
                print("   per-word max rel:", np.array2string(w, precision=2, max_line_width=160))
                print("   env 0 quad:", np.array2string(z[f"{tag}_quad"][0], precision=4, max_line_width=160))
                print("   env 0 lane:", np.array2string(z[f"{tag}_lane"][0], precision=4, max_line_width=160))
    if len(outs) >= 2:
        (la, a), (lb, b) = list(outs.items())[:2]
        for tag in ("zero", "rand"):
            ta, tb = a[f"{tag}_trace"], b[f"{tag}_trace"]
            print(f"-- {tag}: {os.path.basename(la)} vs {os.path.basename(lb)}, per phase (lanes 0..255)")
            for p in range(8):
                for s in range(8):
                    x, y = ta[:, p, s], tb[:, p, s]
                    d = np.abs(x - y) / np.maximum(1.0, np.abs(y))
                    nf = int((~np.isfinite(x)).sum()), int((~np.isfinite(y)).sum())
                    if not (d <= 1e-12).all() or nf != (0, 0):
                        lanes = np.flatnonzero(~(d <= 1e-12))
                        print(f"   phase {p} {PH[p]:13s} {SLOTS[p][s]:8s}: {len(lanes)} lanes differ "
                              f"(first {lanes[:8].tolist()}), non-finite {nf}; lane {lanes[0] if len(lanes) else 0}: "
                              f"{x[lanes[0] if len(lanes) else 0]!r} vs {y[lanes[0] if len(lanes) else 0]!r}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
    else:
        libs = sys.argv[1:] or [os.path.join(REPO, "pybullet-gym_amd", f"libpbg_trace_{v}.so") for v in ("def", "trk", "plain")]
        main(libs)

"""Register-file poison probe of the float64 quad miscompile (dev tool).

For one library: one zero-action and one random-action step of 64 Ant envs (tools/f64_quad_trace.py
--child), each right after every CU's LDS is zeroed and every SIMD's register file is set to
BASE | index (tools/libvgpr_poison.so), for several BASEs, twice each.  A build whose result depends on
the register file's contents reads a register lane it never wrote; with a quiet-NaN BASE the NaN words
of its state carry the index of the register (low 9 bits of the high word: VGPR i -> i, AGPR i ->
0x100 | i).

  python tools/vgpr_poison_probe.py LIB [BASE ...]
  python tools/vgpr_poison_probe.py LIB --bisect [A B]   # the registers whose contents the result depends on:
      register subsets set to A (default 0x3FF00000), the rest to B (0x7FF80000), halved while the result
      differs from the all-B run
"""
import collections
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(HERE)), "gpurun_out")


def run(lib, base, tag):
    out = os.path.join(OUT, f"vgpr_{tag}.npz")
    env = dict(os.environ, PBG_POISON="0x00000000")
    if base:
        env["PBG_VGPR_POISON"] = base
    else:
        env.pop("PBG_VGPR_POISON", None)
    with open(out.replace(".npz", ".log"), "w") as log:
        subprocess.check_call([sys.executable, os.path.join(HERE, "f64_quad_trace.py"), "--child", lib, out], env=env,
                              timeout=120, stdout=log, stderr=subprocess.STDOUT)
    return np.load(out)


def describe(z, tag):
    res = {}
    for step in ("zero", "rand"):
        q, ln = z[f"{step}_quad"], z[f"{step}_lane"]
        rel = (np.abs(q - ln) / np.maximum(1.0, np.abs(ln))).max(axis=1)
        bad = int((~(rel <= 1e-9)).sum())
        words = q.view(np.uint64)
        nan = ~np.isfinite(q)
        hi = (words[nan] >> np.uint64(32)).astype(np.uint32)
        idx = collections.Counter(int(h & 0x1FF) for h in hi if (h & 0xFFF80000) in (0x7FF80000, 0xFFF80000))
        res[step] = (bad, int(nan.sum()), idx.most_common(6))
    print(f"{tag}: " + "; ".join(f"{s} step: {b} of 64 envs above 1e-9, {n} NaN words, NaN high-word "
                                 f"indices {i}" for s, (b, n, i) in res.items()), flush=True)


def same(x, y):
    return all((x[f"{s}_quad"].view(np.uint64) == y[f"{s}_quad"].view(np.uint64)).all() for s in ("zero", "rand"))


def bisect(lib, a, b):
    cnt = [0]

    def run_mask(regs):
        m = np.zeros(16, np.uint32)
        for r in regs:
            m[r >> 5] |= np.uint32(1) << np.uint32(r & 31)
        cnt[0] += 1
        return run(lib, f"{a}:{b}:" + ",".join(f"{int(w):08x}" for w in m), f"mask{cnt[0]}")

    ref = run_mask([])
    ref2 = run_mask([])
    print(f"all-B twice identical: {same(ref, ref2)}", flush=True)
    full = run_mask(range(512))
    print(f"all-A differs from all-B: {not same(full, ref)}; all-A twice identical: {same(full, run_mask(range(512)))}",
          flush=True)
    found = []

    # group test from the all-A side: the registers of S set to B, the rest A; a result unlike the
    # all-A run means S holds a register the kernel reads (a NaN high word in any of the words it
    # combines gives the all-B result, so testing from the all-B side needs every such word at once)
    def rec(regs):
        if cnt[0] >= 160:
            print(f"  run budget spent; unresolved: {regs[0]}..{regs[-1]}", flush=True)
            return
        rs = set(regs)
        z = run_mask([r for r in range(512) if r not in rs])
        if same(z, full):
            return
        if len(regs) == 1:
            r = regs[0]
            found.append(r)
            d = {s: int((z[f"{s}_quad"].view(np.uint64) != full[f"{s}_quad"].view(np.uint64)).sum()) for s in ("zero", "rand")}
            print(f"  sensitive: {'v' if r < 256 else 'a'}{r % 256} (state words changed {d})", flush=True)
            return
        h = len(regs) // 2
        rec(regs[:h])
        rec(regs[h:])

    rec(list(range(512)))
    print(f"sensitive registers: {[('v' if r < 256 else 'a') + str(r % 256) for r in found]} ({cnt[0]} runs)", flush=True)


def main():
    lib = os.path.abspath(sys.argv[1])
    if len(sys.argv) > 2 and sys.argv[2] == "--bisect":
        ab = sys.argv[3:5] if len(sys.argv) >= 5 else ["0x3FF00000", "0x7FF80000"]
        bisect(lib, *ab)
        return
    bases = sys.argv[2:] or ["0x7FF80000", "0x7FFC0000", "0x3FF00000"]
    runs = {}
    runs["none_0"] = run(lib, None, "none_0")
    runs["none_1"] = run(lib, None, "none_1")
    for b in bases:
        for k in range(2):
            runs[f"{b}_{k}"] = run(lib, b, f"{b}_{k}")
    for tag, z in runs.items():
        describe(z, tag)
    keys = list(runs)
    for i, a in enumerate(keys):
        for b in keys[i + 1:]:
            d = {s: int((runs[a][f"{s}_quad"].view(np.uint64) != runs[b][f"{s}_quad"].view(np.uint64)).sum())
                 for s in ("zero", "rand")}
            print(f"  {a} vs {b}: state words differing {d}", flush=True)


if __name__ == "__main__":
    main()

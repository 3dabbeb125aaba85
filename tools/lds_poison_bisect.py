"""Locate the LDS words a kernel build reads without writing them in the launch (the float64 quad
miscompile).  For one library: a baseline step with all of LDS zero, then one
step per word range with only that range NaN-poisoned (tools/liblds_poison.so through
tools/f64_quad_trace.py --child, PBG_POISON_RANGE); a range whose poison changes the quad kernel's
state after the zero-action step holds words the kernel read before writing.

  python tools/lds_poison_bisect.py LIB BEGIN END CHUNKS
  python tools/lds_poison_bisect.py LIB --repeat N     # N runs after all-zero LDS, then 2 after all-NaN:
                                                       # state words differing from the first run
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def run(lib, pattern, rng, tag, trace_tool):
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(HERE)), "gpurun_out", f"bisect_{tag}.npz")
    env = dict(os.environ, PBG_POISON=pattern, PBG_POISON_RANGE=rng)
    subprocess.check_call([sys.executable, trace_tool, "--child", lib, out], env=env, timeout=120,
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return np.load(out)


def main(lib, begin, end, chunks, trace_tool):
    base = run(lib, "0x00000000", "0:0", "base", trace_tool)
    step = max(1, (end - begin + chunks - 1) // chunks)
    for b in range(begin, end, step):
        e = min(end, b + step)
        z = run(lib, "0x7FC00000", f"{b}:{e}", f"{b}_{e}", trace_tool)
        d = {t: int((z[t].view(np.uint64) != base[t].view(np.uint64)).sum()) for t in ("zero_quad", "rand_quad")}
        print(f"words [{b}, {e}): state words changed by the poison: zero step {d['zero_quad']}, "
              f"rand step {d['rand_quad']}", flush=True)


def repeat(lib, n, trace_tool):
    rs = [run(lib, "0x00000000", "0:0", f"rep{i}", trace_tool) for i in range(n)]
    rs += [run(lib, "0x7FC00000", "0:40960", f"repnan{i}", trace_tool) for i in range(2)]
    for i in range(1, len(rs)):
        d = {t: int((rs[i][t].view(np.uint64) != rs[0][t].view(np.uint64)).sum()) for t in ("zero_quad", "rand_quad")}
        print(f"run {i} ({'zero' if i < n else 'NaN'} LDS) vs run 0: {d}", flush=True)


if __name__ == "__main__":
    tt = os.environ.get("PBG_TRACE_TOOL", os.path.join(HERE, "f64_quad_trace.py"))
    if sys.argv[2] == "--repeat":
        repeat(sys.argv[1], int(sys.argv[3]), tt)
    else:
        main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), tt)

"""Did a machine scheduler reorder LDS stores against LDS loads, or memory operations across a
wavefront fence / wave barrier?  (The float64 quad miscompile study)

Dump the kernel's MIR around a scheduler and compare the order of its memory operations per block:

  hipcc ... --cuda-device-only -S -o /dev/null -mllvm -print-before=machine-scheduler \\
      -mllvm -print-after=machine-scheduler -mllvm -filter-print-funcs=<mangled kernel> src.hip 2> mir.txt
  python tools/mir_sched_check.py mir.txt                 # (postmisched: the post-RA scheduler)

Prints, per pair of reordered operations, its kind (ldsW / ldsR / sync / mem) and the totals.
Identical instruction texts are matched by occurrence.
"""
import collections
import re
import sys


def blocks(s):
    out = collections.OrderedDict()
    cur = None
    for line in s.splitlines():
        m = re.match(r"^\s*\d*B?\s*(bb\.\d+)", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        m = re.match(r"^\s*(?:\d+B)?\s+(\S.*)$", line)
        if m and cur and not m.group(1).startswith(("successors", "liveins", "predecessors", ";")):
            out[cur].append(m.group(1).strip())
    return out


def kind(i):
    if any(t in i for t in ("WAVE_BARRIER", "ATOMIC_FENCE", "INLINEASM", "SCHED_BARRIER", "S_BARRIER")):
        return "sync"
    if ":: (" in i and ("(store" in i or "(load" in i):
        if "addrspace 3" in i:
            return "ldsW" if "(store" in i else "ldsR"
        return "mem"
    return None


def tag(lst):
    c = collections.Counter()
    out = []
    for i in lst:
        c[i] += 1
        out.append((i, c[i]))
    return out


def main(path):
    txt = open(path).read()
    parts = re.split(r"^# \*\*\* IR Dump (?:Before|After) .*Machine Instruction Scheduler.*$", txt, flags=re.M)
    B, A = blocks(parts[1]), blocks(parts[2])
    flips = collections.Counter()
    for bb in B:
        if bb not in A:
            continue
        b = tag([i for i in B[bb] if kind(i)])
        a = tag([i for i in A[bb] if kind(i)])
        if set(b) != set(a):  # flags (kill / undef) rewritten: not a reordering
            continue
        pos = {t: k for k, t in enumerate(a)}
        for x in range(len(b)):
            for y in range(x + 1, len(b)):
                if pos[b[x]] > pos[b[y]]:
                    key = (kind(b[x][0]), kind(b[y][0]))
                    flips[key] += 1
                    if "sync" in key or key in (("ldsW", "ldsR"), ("ldsR", "ldsW")):
                        print(bb, key, "|", b[x][0][:120], "||", b[y][0][:120])
    print("reordered pairs by kind:", dict(flips))


if __name__ == "__main__":
    main(sys.argv[1])

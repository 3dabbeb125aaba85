#!/usr/bin/env python3
"""Static use-before-definition check of a kernel's gfx950 ISA (hipcc --cuda-device-only -S output).

For every VGPR / AGPR and every byte of the private (scratch) segment addressed with a constant
offset, a forward must-be-defined data flow over the kernel's basic blocks (intersection at joins,
EXEC ignored: a write under a partial EXEC counts as a definition) reports each instruction that
reads a register or scratch byte which is not written on every path from the kernel's entry
(v0, the packed work-item id, is defined at entry).

Sources of a read: every operand but the first of a defining instruction, every operand of a store,
plus the destination of read-modify-write forms (v_fmac / v_mac, v_writelane, DPP without
bound_ctrl or with a partial row / bank mask, SDWA with dst_unused:UNUSED_PRESERVE, d16_hi loads).

    python tools/isa_uninit.py build/asm/team64_Ant.s [--kernel SUBSTR] [--show N]

Used on the round-5 float64 quad miscompile: the default-schedule build of the
round-5 source against its trackers build and the current source.
"""
import argparse
import re
import sys

REG = re.compile(r"\b([va])(?:(\d+)\b|\[(\d+):(\d+)\])")
LABEL = re.compile(r"^(\.LBB\d+_\d+):")
NOUSE_DST = ("v_cmp", "v_readlane", "v_readfirstlane")


def regs_of(text):
    out = []
    for m in REG.finditer(text):
        base = 0 if m.group(1) == "v" else 256
        if m.group(2) is not None:
            out.append(base + int(m.group(2)))
        else:
            out.extend(base + r for r in range(int(m.group(3)), int(m.group(4)) + 1))
    return out


def split_ops(s):
    """Top-level comma split (quad_perm:[1,0,3,2] keeps its commas)."""
    ops, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def width(mn):
    for suf, w in (("dwordx4", 16), ("dwordx3", 12), ("dwordx2", 8), ("dword", 4), ("short", 2),
                   ("ushort", 2), ("sshort", 2), ("byte", 1), ("ubyte", 1), ("sbyte", 1)):
        if mn.endswith(suf):
            return w
    return 4


def kernels(path):
    """The mangled names of the kernels (function labels) of an ISA file."""
    return [ln.split(":")[0] for ln in open(path).read().split("\n")
            if ln.startswith("_Z") and ":" in ln and "@" in ln]


def parse(path, kernel):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        if ln.startswith("_Z") and ln.split(":")[0].endswith(":") is False and ":" in ln and (kernel in ln):
            start = i
            break
    if start is None:
        sys.exit(f"no kernel matching {kernel!r} in {path}")
    insts = []  # (lineno, label-or-None, mnemonic, operand string, raw)
    for i in range(start + 1, len(lines)):
        ln = lines[i]
        if ln.startswith(".Lfunc_end"):
            break
        m = LABEL.match(ln)
        if m:
            insts.append((i + 1, m.group(1), None, "", ln))
            continue
        if ln.startswith("; %bb."):
            insts.append((i + 1, ln.strip(), None, "", ln))
            continue
        body = ln.split(";")[0].strip()
        if not body or body.startswith("."):
            continue
        parts = body.split(None, 1)
        insts.append((i + 1, None, parts[0], parts[1] if len(parts) > 1 else "", ln.strip()))
    return insts


def analyse(insts):
    # basic blocks
    blocks, cur, names = [], None, {}
    for ins in insts:
        if ins[1] is not None:
            if cur is not None and cur["insts"] or cur is not None:
                blocks.append(cur)
            cur = {"name": ins[1], "insts": []}
            names[ins[1]] = len(blocks)
            continue
        if cur is None:
            cur = {"name": "entry", "insts": []}
            names["entry"] = 0
        cur["insts"].append(ins)
        mn = ins[2]
        if mn.startswith("s_branch") or mn.startswith("s_cbranch") or mn == "s_endpgm" or mn.startswith("s_setpc"):
            blocks.append(cur)
            cur = {"name": f"after{ins[0]}", "insts": []}
            names[cur["name"]] = len(blocks)
    if cur is not None:
        blocks.append(cur)
    blocks = [b for b in blocks]
    names = {b["name"]: k for k, b in enumerate(blocks)}
    succ = [[] for _ in blocks]
    for k, b in enumerate(blocks):
        last = b["insts"][-1] if b["insts"] else None
        mn = last[2] if last else ""
        if mn.startswith("s_branch"):
            succ[k].append(names[last[3].strip()])
        elif mn.startswith("s_cbranch"):
            succ[k].append(names[last[3].strip()])
            if k + 1 < len(blocks):
                succ[k].append(k + 1)
        elif mn == "s_endpgm" or mn.startswith("s_setpc"):
            pass
        elif k + 1 < len(blocks):
            succ[k].append(k + 1)
    pred = [[] for _ in blocks]
    for k, ss in enumerate(succ):
        for s in ss:
            pred[s].append(k)

    def effects(ins):
        """(uses_regs, defs_regs, uses_scratch_bytes, defs_scratch_bytes, note)"""
        _, _, mn, opstr, raw = ins
        ops = split_ops(opstr)
        uses, defs, su, sd, note = [], [], [], [], ""
        if not ops:
            return uses, defs, su, sd, note
        if mn.startswith("scratch_"):
            off = re.search(r"offset:(-?\d+)", opstr)
            o = int(off.group(1)) if off else 0
            w = width(mn)
            if "load" in mn:
                defs = regs_of(ops[0])
                vaddr = regs_of(ops[1]) if len(ops) > 1 else []
                uses = vaddr
                if vaddr:
                    note = "scratch load with a VGPR address (run-time-indexed private memory)"
                else:
                    su = list(range(o, o + w))
            else:
                vaddr = regs_of(ops[0])
                uses = vaddr + regs_of(ops[1])
                if vaddr:
                    note = "scratch store with a VGPR address (run-time-indexed private memory)"
                else:
                    sd = list(range(o, o + w))
            return uses, defs, su, sd, note
        is_store = ("store" in mn) or (mn.startswith("ds_") and not ("read" in mn or "rtn" in mn
                                        or mn.startswith("ds_bpermute") or mn.startswith("ds_permute")
                                        or mn.startswith("ds_swizzle")))
        if mn.startswith("s_") or mn.startswith("buffer_wbl2") or mn.startswith("buffer_inv"):
            uses = regs_of(opstr)  # s_ instructions never name VGPRs; kept for completeness
            return uses, defs, su, sd, note
        if is_store:
            return regs_of(opstr), defs, su, sd, note
        first = regs_of(ops[0])
        rest = regs_of(",".join(ops[1:]))
        if mn.startswith(NOUSE_DST):
            return first + rest, [], su, sd, note
        defs = first
        uses = rest
        rmw = (mn.startswith("v_fmac") or mn.startswith("v_mac") or mn.startswith("v_writelane")
               or "d16_hi" in mn or "UNUSED_PRESERVE" in opstr)
        if "_dpp" in mn:
            full = "row_mask:0xf" in opstr and "bank_mask:0xf" in opstr
            if not (full and "bound_ctrl" in opstr):
                rmw = True
        if mn.startswith("v_swap"):
            rmw = True
        if rmw:
            uses = uses + first
        return uses, defs, su, sd, note

    ALL = (1 << 512) - 1
    SALL = (1 << 4096) - 1
    n = len(blocks)
    din = [ALL] * n
    sin = [SALL] * n
    entry_def = 1 << 0
    din[0] = entry_def
    sin[0] = 0
    eff = [[effects(ins) for ins in b["insts"]] for b in blocks]

    def mask(rs):
        m = 0
        for r in rs:
            m |= 1 << r
        return m

    gen = []
    for k in range(n):
        g = 0
        s = 0
        for (u, d, su, sd, _) in eff[k]:
            g |= mask(d)
            s |= mask(sd)
        gen.append((g, s))
    changed = True
    while changed:
        changed = False
        for k in range(n):
            if k == 0:
                dk, sk = entry_def, 0
            else:
                dk, sk = ALL, SALL
                if not pred[k]:
                    dk, sk = ALL, SALL  # unreachable
                for p in pred[k]:
                    dk &= din[p] | gen[p][0]
                    sk &= sin[p] | gen[p][1]
            if dk != din[k] or sk != sin[k]:
                din[k], sin[k] = dk, sk
                changed = True
    reports = []
    for k in range(n):
        if k != 0 and not pred[k]:
            continue
        d, s = din[k], sin[k]
        for ins, (u, df, su, sd, note) in zip(blocks[k]["insts"], eff[k]):
            bad = [r for r in u if not (d >> r) & 1]
            sbad = [b for b in su if not (s >> b) & 1]
            if bad or sbad or note:
                reports.append((ins[0], ins[4], bad, sbad, note))
            d |= mask(df)
            s |= mask(sd)
    return blocks, reports


COPY = ("v_accvgpr_write_b32", "v_accvgpr_read_b32", "v_mov_b32_e32", "v_mov_b32", "v_accvgpr_mov_b32",
        "v_mov_b64_e32", "v_mov_b64")


def exec_copies(insts):
    """Copies of a live-through value placed under a partial EXEC: a register move (or a spill to a
    constant-offset scratch slot) in the join block of a
    divergent region (after its last label, before the `s_or_b64 exec, exec, sN` that ends the region)
    whose source was last written before the region's `s_and_saveexec_b64 sN` and whose destination is
    read after the region before it is written again.  The move copies only the lanes inside the
    region; the other lanes read the destination's stale contents (the round-5 float64 quad
    miscompile)."""
    code = [i for i in insts]
    stack, out = [], []
    label_at = {c[1]: t for t, c in enumerate(code) if c[1] is not None and c[1].startswith(".LBB")}
    branches = [(t, c[3].strip()) for t, c in enumerate(code) if c[2] and c[2].startswith(("s_branch", "s_cbranch"))]

    def sese(a, b):
        """Single entry, single exit: no branch inside [a, b] leaves it (other than to the label right
        after b) and no branch from outside targets a label strictly inside it."""
        for t, tgt in branches:
            d = label_at.get(tgt)
            if d is None:
                continue
            inside_src, inside_dst = a < t < b, a < d < b
            if inside_src and not inside_dst and d != b + 1:
                return False
            if not inside_src and inside_dst:
                return False
        return True
    last_label = 0
    for k, (ln, lab, mn, ops, raw) in enumerate(code):
        if lab is not None:
            last_label = k
            continue
        o = ops.replace(" ", "")
        if mn == "s_and_saveexec_b64":
            stack.append((o.split(",")[0], k))
        elif mn == "s_xor_b64" and stack and o.split(",")[1:] == ["exec", stack[-1][0]]:
            stack[-1] = (o.split(",")[0], stack[-1][1])  # if / else: the else lanes' mask ends the region
        elif mn == "s_or_b64" and o.startswith("exec,exec,"):
            sp = o.split(",")[2]
            at = [i for i, (r, _) in enumerate(stack) if r == sp]
            if not at:
                continue  # a loop's exit mask or an else arm: no s_and_saveexec of this pair is open
            _, start = stack[at[-1]]
            del stack[at[-1]:]
            if not sese(start, k):
                continue  # an unstructured region (branches in or out): its lanes are not one mask
            for j in range(max(last_label, start) + 1, k):
                jl, _, jmn, jops, jraw = code[j]
                parts = split_ops(jops)
                slot = None
                if jmn.startswith("scratch_store") and len(parts) >= 2 and not regs_of(parts[0]):
                    # a spill of a live-through value under the region's EXEC (constant-offset slot)
                    m = re.search(r"offset:(-?\d+)", jops)
                    slot = set(range(int(m.group(1)) if m else 0, (int(m.group(1)) if m else 0) + width(jmn)))
                    dst, src = [], regs_of(parts[1])
                elif jmn in COPY:
                    dst, src = regs_of(parts[0]), regs_of(",".join(parts[1:]))
                    if not dst:
                        continue
                else:
                    continue
                if not src:
                    continue
                # the source's last write before the copy
                sdef = None
                for t in range(j - 1, -1, -1):
                    tm = code[t][2]
                    if tm is None:
                        continue
                    tops = split_ops(code[t][3])
                    if tops and not tm.startswith(("s_", "v_cmp", "v_readlane", "v_readfirstlane")) and "store" not in tm \
                            and not (tm.startswith("ds_") and "read" not in tm) and set(regs_of(tops[0])) & set(src):
                        sdef = t
                        break
                if sdef is None or sdef >= start:
                    continue
                # the destination read after the region before a rewrite
                for t in range(k + 1, len(code)):
                    tm = code[t][2]
                    if tm is None:
                        continue
                    tops = split_ops(code[t][3])
                    if not tops:
                        continue
                    if slot is not None:
                        if tm.startswith("scratch_") and len(tops) >= 2:
                            m = re.search(r"offset:(-?\d+)", code[t][3])
                            o = int(m.group(1)) if m else 0
                            bytes_ = set(range(o, o + width(tm)))
                            if "load" in tm and not regs_of(tops[1]) and bytes_ & slot:
                                out.append((jl, jraw, code[sdef][0], code[start][0], code[k][0], code[t][0], code[t][4]))
                                break
                            if "store" in tm and not regs_of(tops[0]) and bytes_ >= slot:
                                break
                        continue
                    defines = not tm.startswith(("s_", "v_cmp", "v_readlane", "v_readfirstlane")) and "store" not in tm \
                        and not (tm.startswith("ds_") and "read" not in tm)
                    reads = set(regs_of(",".join(tops[1:] if defines else tops)))
                    if reads & set(dst):
                        out.append((jl, jraw, code[sdef][0], code[start][0], code[k][0], code[t][0], code[t][4]))
                        break
                    if defines and set(regs_of(tops[0])) >= set(dst):
                        break
    return out


def rname(r):
    return f"v{r}" if r < 256 else f"a{r - 256}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="team_step_kernelINS_3F64IN10pbg_models3AntE")
    ap.add_argument("--show", type=int, default=40)
    ap.add_argument("--exec-copies", action="store_true", help="only the partial-EXEC copy check; exit 1 on a hit")
    ap.add_argument("--all", action="store_true", help="--exec-copies over every kernel of the file")
    a = ap.parse_args()
    if a.all:
        names = kernels(a.asm)
        hits = 0
        for k in names:
            ec = exec_copies(parse(a.asm, k))
            hits += len(ec)
            print(f"{k[:110]}: {len(ec)} partial-EXEC copies read after their region")
            for jl, raw, sdef, start, end, rl, rraw in ec[: a.show]:
                print(f"  line {jl}: {raw}   (source written at line {sdef}, region {start}..{end}, read at line {rl}: {rraw})")
        print(f"{a.asm}: {len(names)} kernels, {hits} partial-EXEC copies")
        sys.exit(1 if hits else 0)
    insts = parse(a.asm, a.kernel)
    ec = exec_copies(insts)
    print(f"{a.asm}: {len(ec)} copies of a live-through value under a region's partial EXEC, read after the region")
    for jl, raw, sdef, start, end, rl, rraw in ec[: a.show]:
        print(f"  line {jl}: {raw}   (source written at line {sdef}, region {start}..{end}, read at line {rl}: {rraw})")
    if a.exec_copies:
        sys.exit(1 if ec else 0)
    blocks, reps = analyse(insts)
    nin = sum(1 for i in insts if i[2])
    print(f"{a.asm}: {nin} instructions, {len(blocks)} blocks, {len(reps)} reads of a register / scratch "
          f"byte not defined on every path from the entry")
    for ln, raw, bad, sbad, note in reps[: a.show]:
        what = []
        if bad:
            what.append("regs " + ",".join(rname(r) for r in bad))
        if sbad:
            what.append(f"scratch bytes {min(sbad)}..{max(sbad)}")
        if note:
            what.append(note)
        print(f"  line {ln}: {raw}    <- {'; '.join(what)}")


if __name__ == "__main__":
    main()

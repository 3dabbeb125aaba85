"""Count instructions matching a prefix per source line in a -gline-tables-only .s (dev tool).

usage: python tools/isa_lines.py file.s [kernel-substring] [instr-prefix]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split('\n')
kern = sys.argv[2] if len(sys.argv) > 2 else 'step_kernel'
pre = sys.argv[3] if len(sys.argv) > 3 else 'v_cndmask'
files = {}
for l in s:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
cur, inside, first, c = None, False, None, collections.Counter()
for l in s:
    if re.match(r'^_Z\w+:', l):
        inside = kern in l and (first is None or first == l)
        if inside:
            first = l
    if not inside:
        continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = (files.get(m.group(1)), int(m.group(2)))
    elif l.startswith('\t') and l.strip().startswith(pre):
        c[cur] += 1
for k, v in c.most_common(25):
    print(k, v)

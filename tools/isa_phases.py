"""Per-phase instruction mix of a -DPBG_STAMPS build's .s (segments between s_memtime)."""
import re, sys
s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
starts = [i for i, l in enumerate(s) if re.match(r'^_Z\w+:', l)]
for k, i in enumerate(starts):
    name = s[i].split(':')[0]
    if pat not in name:
        continue
    end = starts[k + 1] if k + 1 < len(starts) else len(s)
    body = [l.strip() for l in s[i:end] if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    seg, segs = [], []
    for l in body:
        if l.startswith('s_memtime'):
            segs.append(seg); seg = []
        else:
            seg.append(l)
    segs.append(seg)
    print(name[-50:])
    for j, sg in enumerate(segs):
        c = lambda p: sum(1 for l in sg if l.startswith(p))
        print(f"  seg {j:2d}: instr {len(sg):6d} scratch_ld {c('scratch_load'):4d} scratch_st {c('scratch_store'):4d} "
              f"ds {c('ds_'):4d} glb {c('global_'):4d} accvgpr {sum('accvgpr' in l for l in sg):5d} valu {c('v_'):6d}")

"""Instruction-class counts per kernel in a hipcc --save-temps .s file (dev tool)."""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2] if len(sys.argv) > 2 else 'step_kernel'
starts = [i for i, l in enumerate(s) if re.match(r'^_Z\w+:', l)]
for k, i in enumerate(starts):
    name = s[i].split(':')[0]
    if pat not in name:
        continue
    end = starts[k + 1] if k + 1 < len(starts) else len(s)
    body = [l.strip() for l in s[i:end] if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    cnt = lambda p: sum(1 for l in body if l.startswith(p))
    print(f"{name[-45:]:45s} instr {len(body):6d} scratch_ld {cnt('scratch_load'):5d} scratch_st {cnt('scratch_store'):5d} "
          f"glb_ld {cnt('global_load'):4d} glb_st {cnt('global_store'):4d} ds {cnt('ds_'):4d} valu {cnt('v_'):6d} salu {cnt('s_'):5d} "
          f"f64 {sum(('_f64' in l) for l in body):4d}")

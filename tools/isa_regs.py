"""Per-kernel register / scratch metadata of a hipcc -S .s file (dev tool).

usage: python tools/isa_regs.py build/asm/robot_Humanoid.s [kernel-substring]
"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in s.split("\n  - ")[1:]:
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or pat not in m.group(1) or "kernel" not in m.group(1):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{m.group(1)[-70:]:70s} vgpr {g('vgpr_count'):>4s} agpr {g('agpr_count'):>4s} "
          f"vspill {g('vgpr_spill_count'):>4s} sspill {g('sgpr_spill_count'):>4s} scratch {g('private_segment_fixed_size'):>5s}")

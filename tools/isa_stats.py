"""Instruction mix of kernels in build/wpt_render.s (make asm): total, VALU,
SALU, global loads, branches, per mangled-name fragment.
Usage: python tools/isa_stats.py FRAG [FRAG ...]"""
import re
import sys

s = open(sys.argv[1] if sys.argv[1].endswith(".s") else "wasm-pathtracer_amd/csrc/build/wpt_render.s").read()
frags = [a for a in sys.argv[1:] if not a.endswith(".s")]
for frag in frags:
    m = re.search(r"^(_ZN\S*" + re.escape(frag) + r"\S*):", s, re.M)
    if not m:
        print(frag, "not found")
        continue
    end = s.index(".Lfunc_end", m.end())
    lines = [l.strip() for l in s[m.end():end].split("\n")]
    ins = [l for l in lines if l and not l.startswith((".", ";")) and not l.endswith(":") and ":" not in l.split()[0]]
    cnt = lambda p: sum(1 for l in ins if l.startswith(p))
    print(f"{frag:28s} insts {len(ins):5d} valu {cnt('v_'):5d} salu {cnt('s_'):5d} "
          f"gload {sum(1 for l in ins if 'global_load' in l):3d} ds {cnt('ds_'):3d} branch {cnt('s_cbranch'):4d}")

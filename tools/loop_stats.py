"""Instruction mix of a kernel's outermost loop (blocks annotated 'in Loop:
Header=<H>' plus nested loops) in build/wpt_render.s. Usage:
python tools/loop_stats.py FILE.s FRAG [FRAG ...]"""
import re
import sys

s = open(sys.argv[1]).read()
for frag in sys.argv[2:]:
    m = re.search(r"^(_ZN\S*" + re.escape(frag) + r"\S*):", s, re.M)
    end = s.index(".Lfunc_end", m.end())
    body = s[m.end():end].split("\n")
    # outermost loop header: the first 'Loop Header: Depth=1'
    blocks, cur, hdr = {}, None, None
    parent = {}
    for line in body:
        mb = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)$", line.strip()) or re.match(r"^(\.LBB\d+_\d+):(.*)", line)
        if mb:
            cur = mb.group(1)
            blocks[cur] = []
            note = mb.group(2)
            mh = re.search(r"Loop Header: Depth=1", note)
            if mh and hdr is None:
                hdr = cur
            mi = re.search(r"Header=(\S+) Depth=(\d+)", note)
            parent[cur] = ("LBB" + mi.group(1)[2:]) if mi else None
            if mh:
                parent[cur] = cur
            continue
        if line.strip().startswith("; %bb."):
            cur = line.strip().split(":")[0]
            blocks[cur] = []
            mi = re.search(r"Header=(\S+) Depth=(\d+)", line)
            parent[cur] = ("LBB" + mi.group(1)[2:]) if mi else None
            continue
        t = line.strip()
        if cur and t and not t.startswith((";", ".")):
            blocks[cur].append(t)
    # blocks belonging to the outer loop: annotated with Depth>=1 (any header nested in it)
    inloop = [b for b in blocks if b == hdr or (parent.get(b) is not None)]
    ins = [i for b in inloop for i in blocks[b]]
    c = lambda p: sum(1 for i in ins if i.startswith(p))
    print(f"{frag:26s} loop blocks {len(inloop):4d} insts {len(ins):5d} valu {c('v_'):5d} salu {c('s_'):5d} "
          f"vmem {sum(1 for i in ins if i.startswith(('global_', 'buffer_', 'flat_'))):3d} ds {c('ds_'):3d} "
          f"waitcnt {c('s_waitcnt'):4d} cbranch {c('s_cbranch'):4d}")

"""Per-body instruction table of a traversal kernel.

Attributes every instruction of one kernel instantiation in
`build/wpt_render_g.s` (`make asmg`: the production flags plus source-line
tables) to the body of the traversal loop its source line belongs to:

  expand  both children of an internal node: the pair load, the two slab
          tests, the push of the farther child (`step`'s internal-node branch,
          `expand_pair`, `box_entry`, `push`, `encode_child`, `stack_store`)
  leaf    one leaf's primitives (`leaf_test`, the triangle / shape tests)
  pop     resuming the deepest uncull'd entry (`pop`, `pop_top`, `stack_load`)
  refill  idle lanes taking rays from the wave's feed and starting them
          (`WaveFeed`, `begin_extend` / `begin_shadow`, `enter_root`, the plane
          scan, the hit store)
  loop    the kernel's own loop lines (ballots, exit test, hand-offs) and
          `step`'s leaf-batching decision
  setup   block prologue (`load_hot`: root node, light records, LDS treelet)

Instructions whose line lies in a header (ballot / popcount intrinsics) or
carries no line (compiler-made moves) count for the body of the preceding
attributed instruction. Counts are STATIC (every path through a body, its
rare branches included). With a bench line (`--bench line.json`, from a run
whose `work` block was counted) the table adds how often the loop runs each
body: wave-level executions per ray and lanes per execution (device ballots,
`BodyLanes` in wpt_render.hip; extension and shadow walks together).

Usage: python tools/body_table.py [--kernel k_extendILb1ELb0ELi0E] [--bench line.json]
"""
import argparse
import json
import os
import re
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "wasm-pathtracer_amd", "csrc")

BODIES = ("expand", "leaf", "pop", "refill", "loop", "setup", "other")
FUNCS = {
    "expand": ["expand_pair", "box_entry", "push", "encode_child", "stack_store"],
    "leaf": ["leaf_test", "tri_hit_r", "tri_hit", "prim_hit", "aarect_hit", "aarect_slab", "sphere_roots",
             "plane_hit_leaf"],
    "pop": ["pop", "pop_top", "stack_load"],
    "refill": ["begin_extend", "begin_shadow", "enter_root", "planes_closest", "plane_hit", "inv_dir", "ld3",
               "st_hit", "linear_closest"],
    "setup": ["load_hot"],
}


def func_ranges(src_lines):
    """name -> (first, last) source line (1-based) of each device function
    defined at the top level, by brace matching from its signature line."""
    out = {}
    sig = re.compile(r"^(?:template <[^>]*>\s*)?(?:__device__|__global__|struct)\b")
    i = 0
    n = len(src_lines)
    while i < n:
        m = sig.match(src_lines[i])
        names = [x for x in re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*[({]", src_lines[i])
                 if x not in ("__launch_bounds__", "__attribute__")]
        if not m or not names:
            i += 1
            continue
        name = names[0]
        depth, started, j = 0, False, i
        while j < n:
            for ch in src_lines[j]:
                if ch == "{":
                    depth += 1
                    started = True
                elif ch == "}":
                    depth -= 1
            if started and depth <= 0:
                break
            j += 1
        out.setdefault(name, (i + 1, j + 1))
        i = j + 1
    return out


def kernel_regions(src_lines, kname):
    """Line ranges inside the kernel body: the refill block, the loop, setup."""
    fr = func_ranges(src_lines)
    k0, k1 = fr[kname]
    loop0 = next(i for i in range(k0, k1) if re.search(r"for \(;;\)", src_lines[i - 1]))
    refill0 = next(i for i in range(loop0, k1) if "feed.more()" in src_lines[i - 1] and "nidle" in src_lines[i - 1])
    # the refill block ends at the brace closing its `if`
    depth, j = 0, refill0
    while True:
        depth += src_lines[j - 1].count("{") - src_lines[j - 1].count("}")
        if depth <= 0 and j > refill0:
            break
        j += 1
    return fr, (k0, loop0 - 1), (refill0, j), (loop0, k1)


def classify(fr, kname, setup, refill, loop, step_rng, step_expand, gate=None):
    table = []
    if gate:
        table.append((gate, "loop"))
    for body, names in FUNCS.items():
        for nm in names:
            if nm in fr:
                table.append((fr[nm], body))
    for nm in ("WaveFeed",):
        if nm in fr:
            table.append((fr[nm], "refill"))
    for nm in ("probe_now", "probe_close", "work_add", "work_add_wave", "wave_sum", "BodyLanes"):
        if nm in fr:
            table.append((fr[nm], "other"))
    table.append((step_expand, "expand"))
    table.append((step_rng, "pop"))        # step's remaining lines: the leaf call and the pop
    table.append((refill, "refill"))
    table.append((setup, "setup"))
    table.append((loop, "loop"))

    def body_of(line):
        best = None
        for (a, b), body in table:
            if a <= line <= b and (best is None or (b - a) < best[0]):
                best = (b - a, body)
        return best[1] if best else None
    return body_of


def kind(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_extendILb1ELb0ELi0E")
    ap.add_argument("--asm", default=os.path.join(CSRC, "build", "wpt_render_g.s"))
    ap.add_argument("--bench", default=None)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    src = open(os.path.join(CSRC, "wpt_render.hip")).read().split("\n")
    kname = re.match(r"(k_[a-z0-9_]+?)I", a.kernel).group(1) if "I" in a.kernel else a.kernel
    fr, setup, refill, loop = kernel_regions(src, kname)
    s0, s1 = fr["step"]
    e0 = next(i for i in range(s0, s1) if "if (L.cnt == 0)" in src[i - 1])
    depth, e1 = 0, e0
    while True:
        depth += src[e1 - 1].count("{") - src[e1 - 1].count("}")
        if depth <= 0 and e1 > e0:
            break
        e1 += 1
    # the leaf-batching decision (two ballots and a compare) is loop control
    gate = None
    g0 = next((i for i in range(e1, s1) if "if (LB && TRI_ONLY)" in src[i - 1]), None)
    if g0:
        depth, g1 = 0, g0
        while True:
            depth += src[g1 - 1].count("{") - src[g1 - 1].count("}")
            if depth <= 0 and g1 > g0:
                break
            g1 += 1
        gate = (g0, g1)
    body_of = classify(fr, kname, setup, refill, loop, (s0, s1), (e0, e1), gate)

    s = open(a.asm).read()
    m = re.search(r"^(_ZN\S*" + re.escape(a.kernel) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"{a.kernel} not found in {a.asm} (make asmg)")
    end = s.index(".Lfunc_end", m.end())
    files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
    cur_body, cur_line = "setup", None
    counts = defaultdict(Counter)
    for raw in s[m.end():end].split("\n"):
        t = raw.strip()
        mm = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if mm:
            fname = files.get(mm.group(1), "").split("/")[-1]
            line = int(mm.group(2))
            if fname == "wpt_render.hip" and line > 0:
                b = body_of(line)
                if b:
                    cur_body = b
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        k = kind(t)
        counts[cur_body][k] += 1
        counts[cur_body]["all"] += 1

    rows = []
    tot = Counter()
    for b in BODIES:
        c = counts.get(b)
        if not c:
            continue
        tot.update(c)
        rows.append({"body": b, **{k: c.get(k, 0) for k in ("all", "valu", "salu", "vmem", "lds", "branch", "wait")}})
    rows.append({"body": "total", **{k: tot.get(k, 0) for k in ("all", "valu", "salu", "vmem", "lds", "branch", "wait")}})

    dyn = None
    if a.bench:
        d = json.load(open(a.bench))
        w = d.get("work") or {}
        dyn = {k: w.get(k) for k in ("ext_steps_per_ray", "ext_loop_live_frac", "sh_steps_per_ray", "node_visits_per_ray",
                                     "prim_tests_per_ray", "lanes_per_expand_body", "lanes_per_leaf_body",
                                     "lanes_per_body", "expand_bodies_per_ray", "leaf_bodies_per_ray",
                                     "wave_iters_per_ray")}
    if a.json:
        print(json.dumps({"kernel": a.kernel, "static": rows, "executed": dyn}, indent=1))
        return
    print(f"{a.kernel}: static instructions per loop body (make asmg; every path of a body counted)")
    print(f"| body | all | VALU | SALU | VMEM | LDS | branch | waitcnt |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['body']} | {r['all']} | {r['valu']} | {r['salu']} | {r['vmem']} | {r['lds']} | {r['branch']} | {r['wait']} |")
    if dyn:
        print("executed (device ballots, extension + shadow walks):", json.dumps(dyn))


if __name__ == "__main__":
    main()

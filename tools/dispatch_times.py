"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace CSV, in
launch order, grouped by kernel, plus each kernel's BUSY time: the union of
its dispatch intervals (the renderer's lanes run a kernel's dispatches
concurrently; bench.py's roofline counts one logical launch per bounce whose
duration is that union).

Usage: tools/dispatch_times.py <rocprof output dir> [logical launches per kernel, e.g. k_extend=16]
"""
import csv
import glob
import json
import re
import sys


def load(d):
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
            name = m.group(1).replace(" ", "") if m else r["Kernel_Name"][:40]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def union_ms(iv):
    busy, lo, hi = 0, None, None
    for a, b in sorted(iv):
        if hi is None or a > hi:
            if hi is not None:
                busy += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    if hi is not None:
        busy += hi - lo
    return busy / 1e6


def main():
    rows = load(sys.argv[1])
    logical = dict(a.split("=") for a in sys.argv[2:])
    by = {}
    for a, b, n in rows:
        by.setdefault(n, []).append((a, b))
    out = {}
    for n, iv in by.items():
        durs = [(b - a) / 1e6 for a, b in iv]
        busy = union_ms(iv)
        out[n] = {"dispatches": len(iv), "sum_ms": round(sum(durs), 3), "avg_dispatch_ms": round(sum(durs) / len(iv), 4),
                  "busy_ms": round(busy, 3)}
        if n in logical:
            out[n]["logical_launches"] = int(logical[n])
            out[n]["busy_ms_per_logical_launch"] = round(busy / int(logical[n]), 4)
        print(f"{n:24s} n={len(iv):3d} sum={sum(durs):8.2f} busy={busy:8.2f} ms  "
              + " ".join(f"{x:.2f}" for x in durs[:48]), file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

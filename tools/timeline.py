"""GPU timeline of a rocprofv3 --kernel-trace run: wall span from the first
dispatch start to the last end, the union of all dispatch intervals (GPU
busy), the idle gaps between them (count, total, by size) and each kernel's
own union ("busy") and summed dispatch time. Usage: tools/timeline.py <dir> [t0_ms t1_ms]"""
import csv
import glob
import json
import re
import sys


def load(d):
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+|rocprim|copyBuffer|fillBuffer)", r["Kernel_Name"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30]))
    rows.sort()
    return rows


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main():
    rows = load(sys.argv[1])
    if len(sys.argv) > 3:
        t0 = rows[0][0] + float(sys.argv[2]) * 1e6
        t1 = rows[0][0] + float(sys.argv[3]) * 1e6
        rows = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    u = union([(a, b) for a, b, _ in rows])
    span = (u[-1][1] - u[0][0]) / 1e6
    busy = sum(b - a for a, b in u) / 1e6
    gaps = [(u[i + 1][0] - u[i][1]) / 1e3 for i in range(len(u) - 1)]
    bins = {"<10us": 0, "10-100us": 0, "0.1-1ms": 0, ">1ms": 0}
    tot = {k: 0.0 for k in bins}
    for g in gaps:
        k = "<10us" if g < 10 else "10-100us" if g < 100 else "0.1-1ms" if g < 1000 else ">1ms"
        bins[k] += 1
        tot[k] += g / 1e3
    per = {}
    for a, b, n in rows:
        per.setdefault(n, []).append((a, b))
    kern = {n: {"dispatches": len(iv), "busy_ms": round(sum(y - x for x, y in union(iv)) / 1e6, 2),
                "sum_ms": round(sum(y - x for x, y in iv) / 1e6, 2)} for n, iv in per.items()}
    print(json.dumps({"span_ms": round(span, 2), "gpu_busy_ms": round(busy, 2), "idle_ms": round(span - busy, 2),
                      "gaps": {k: {"count": bins[k], "ms": round(tot[k], 2)} for k in bins},
                      "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["busy_ms"]))}, indent=1))


if __name__ == "__main__":
    main()

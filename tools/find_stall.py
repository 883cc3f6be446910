"""Longest kernels and longest GPU-idle gaps of a rocprofv3 --kernel-trace
run, with the dispatches either side of each gap (what the GPU waited on).
usage: python tools/find_stall.py <trace dir> [--top 8]"""
import argparse
import csv
import glob
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(a.trace + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+|rocprim\w*|copyBuffer\w*|fillBuffer\w*)", r["Kernel_Name"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         m.group(1) if m else r["Kernel_Name"][:40], int(r.get("Grid_Size", 0) or 0)))
    rows.sort()
    t0 = rows[0][0]
    print(f"{len(rows)} dispatches over {(rows[-1][1] - t0) / 1e6:.1f} ms")
    print("longest kernels:")
    for x, y, q, n, g in sorted(rows, key=lambda r: r[0] - r[1])[:a.top]:
        print(f"  {(y - x) / 1e6:10.3f} ms  at {(x - t0) / 1e6:10.1f} ms  q={q} {n} grid={g}")
    end = rows[0][1]
    gaps = []
    for i in range(1, len(rows)):
        if rows[i][0] > end:
            gaps.append((rows[i][0] - end, i))
        end = max(end, rows[i][1])
    print("longest idle gaps:")
    for d, i in sorted(gaps, reverse=True)[:a.top]:
        b = rows[max(0, i - 3):i]
        nx = rows[i:i + 3]
        print(f"  {d / 1e6:10.3f} ms  at {(rows[i][0] - t0) / 1e6:10.1f} ms")
        for x, y, q, n, g in b:
            print(f"      before q={q} {n} grid={g} {(y - x) / 1e3:.1f} us")
        for x, y, q, n, g in nx:
            print(f"      after  q={q} {n} grid={g} {(y - x) / 1e3:.1f} us")


if __name__ == "__main__":
    main()

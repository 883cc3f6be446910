"""Where a session's GPU time goes, per hardware queue, from a rocprofv3
--kernel-trace run (tools/profile_init.sh). The window is the last
`--calls` compute calls' span, found as the trace after the longest idle gap
of the warm-up (or the whole trace with --all). Per queue: the busy time
(union of its dispatch intervals) and the kernels in it; GPU-wide: the time
with 0, 1, 2, 3 and 4+ queues running a kernel, and per kernel kind the
time during which it is the only one running.

usage: python tools/init_phases.py <trace dir> [--skip-ms T] [--bins 2.0]"""
import argparse
import csv
import glob
import json
import re


def load(d):
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+|rocprim\w*|copyBuffer|fillBuffer)", r["Kernel_Name"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         m.group(1) if m else r["Kernel_Name"][:30]))
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
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ms", type=float, default=-1.0,
                    help="start of the window after the first dispatch (default: after the longest gap)")
    ap.add_argument("--bins", type=float, default=2.0, help="ms per bin of the time series")
    a = ap.parse_args()
    rows = load(a.trace)
    if a.skip_ms >= 0:
        t0 = rows[0][0] + a.skip_ms * 1e6
    else:
        # the timed calls follow the longest host gap (session setup, warm-up, clear_stats)
        u = union([(x, y) for x, y, _, _ in rows])
        gaps = [(u[i + 1][0] - u[i][1], u[i + 1][0]) for i in range(len(u) - 1)]
        t0 = max(gaps)[1] if gaps else rows[0][0]
    rows = [r for r in rows if r[0] >= t0]
    t1 = max(r[1] for r in rows)
    span = (t1 - t0) / 1e6
    queues = {}
    for x, y, q, n in rows:
        queues.setdefault(q, []).append((x, y, n))
    per_q = {}
    for q, iv in sorted(queues.items()):
        kinds = {}
        for x, y, n in iv:
            kinds.setdefault(n, []).append((x, y))
        per_q[str(q)] = {"busy_ms": round(sum(y - x for x, y in union([(x, y) for x, y, _ in iv])) / 1e6, 2),
                         "kernels": {n: {"n": len(v), "busy_ms": round(sum(y - x for x, y in union(v)) / 1e6, 2)}
                                     for n, v in sorted(kinds.items(), key=lambda kv: -len(kv[1]))[:8]}}
    # concurrency: sweep the dispatch edges
    ev = []
    for x, y, q, n in rows:
        ev.append((x, 1, q, n))
        ev.append((y, -1, q, n))
    ev.sort()
    active = {}
    conc = {}
    alone = {}
    last = t0
    for t, d, q, n in ev:
        dt = (t - last) / 1e6
        if dt > 0:
            nq = len({qq for (qq, _), c in active.items() if c > 0})
            conc[min(nq, 4)] = conc.get(min(nq, 4), 0.0) + dt
            live = [k for k, c in active.items() if c > 0]
            if len(live) == 1:
                alone[live[0][1]] = alone.get(live[0][1], 0.0) + dt
        last = t
        active[(q, n)] = active.get((q, n), 0) + d
    # time series: per bin, the busy fraction of each queue
    nb = int(span / a.bins) + 1
    series = {str(q): [0.0] * nb for q in queues}
    for q, iv in queues.items():
        for x, y in union([(x, y) for x, y, _ in iv]):
            bx = (x - t0) / 1e6
            by = (y - t0) / 1e6
            while bx < by:
                k = int(bx / a.bins)
                e = min(by, (k + 1) * a.bins)
                series[str(q)][k] += (e - bx) / a.bins
                bx = e
    print(json.dumps({"window_ms": round(span, 2), "dispatches": len(rows),
                      "queues_running_ms": {str(k): round(v, 2) for k, v in sorted(conc.items())},
                      "alone_ms": {k: round(v, 2) for k, v in sorted(alone.items(), key=lambda kv: -kv[1])},
                      "per_queue": per_q,
                      "series_bin_ms": a.bins,
                      "series": {q: [round(v, 2) for v in s] for q, s in series.items()}}, indent=1))


if __name__ == "__main__":
    main()

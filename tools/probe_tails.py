"""Per-launch anatomy of the persistent traversal kernels:
how long each launch runs with few of its waves still alive.

Runs a bench-shaped session with the wave probe on (WPT_OPT_PROBE: every wave
of a traversal launch records its start, the moment its work feed ran dry and
its end on the steady clock), then summarises per kernel kind:
  * launches, summed launch time D (first wave start .. last wave end);
  * wave_live_frac: sum of wave lifetimes / (waves x D);
  * below25: time with fewer than 25 % of the launch's waves alive, and
    dry: time from the first wave whose feed ran dry to the launch end.

Usage on the GPU box: python tools/probe_tails.py [c5|c3|defaults] [launches] [name=value,...] > out.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KIND = {1: "extend", 3: "shadow", 5: "trace"}


def launch_stats(rec, tpu):
    """One launch's wave records (start, dry, end, rays) -> dict (microseconds)."""
    s = rec[:, 0].astype(np.int64)
    e = rec[:, 2].astype(np.int64)
    dry = rec[:, 1].astype(np.int64)
    t0 = s.min()
    # unwrap the 32-bit clock relative to the launch start
    s, e, dry = (s - t0) % (1 << 32), (e - t0) % (1 << 32), (dry - t0) % (1 << 32)
    D = e.max()
    W = len(e)
    life = (e - s).sum()
    # live-wave count over time: +1 at start, -1 at end
    ts = np.concatenate([s, e])
    dv = np.concatenate([np.ones(W, np.int64), -np.ones(W, np.int64)])
    o = np.argsort(ts, kind="stable")
    ts, live = ts[o], np.cumsum(dv[o])
    seg = np.diff(np.append(ts, D))
    below = seg[live < 0.25 * W].sum()
    took = rec[:, 3] > 0
    first_dry = dry[took].min() if took.any() else D
    lives = np.sort((e - s)[took]) if took.any() else np.zeros(1, np.int64)
    return {"D": D / tpu, "waves": W, "life_frac": life / max(W * D, 1), "below25": below / tpu,
            "dry": (D - first_dry) / tpu, "rays": int(rec[:, 3].sum()),
            # lifetimes of the waves that took rays: median, 90th percentile, longest
            "life_p50": float(lives[len(lives) // 2]) / tpu, "life_p90": float(lives[(9 * len(lives)) // 10]) / tpu,
            "life_max": float(lives[-1]) / tpu, "working_waves": int(took.sum())}


def gpu_wide(meta, rec, tpu, capacity):
    """All probed launches on one clock: the traversal waves alive over time
    across every lane's launches (they overlap), against the resident
    capacity of the traversal grid (capacity waves). Returns the share of the
    probed span with fewer than 25 % / 50 % of capacity alive, and the mean."""
    s = np.concatenate([rec[m[4]:m[4] + m[3], 0] for m in meta]).astype(np.int64)
    e = np.concatenate([rec[m[4]:m[4] + m[3], 2] for m in meta]).astype(np.int64)
    t0 = s.min()
    s, e = (s - t0) % (1 << 32), (e - t0) % (1 << 32)
    ts = np.concatenate([s, e])
    dv = np.concatenate([np.ones(len(s), np.int64), -np.ones(len(e), np.int64)])
    o = np.argsort(ts, kind="stable")
    ts, live = ts[o], np.cumsum(dv[o])
    seg = np.diff(np.append(ts, ts[-1]))
    span = ts[-1] - ts[0]
    return {"span_us": float(span / tpu), "mean_live_frac": float((live * seg).sum() / max(span, 1) / capacity),
            "below25_frac": float(seg[live < 0.25 * capacity].sum() / max(span, 1)),
            "below50_frac": float(seg[live < 0.5 * capacity].sum() / max(span, 1)),
            "capacity_waves": int(capacity)}


def summarise(meta, rec, tpu):
    out = {}
    for kind in sorted(set(meta[:, 0].tolist())):
        rows = [launch_stats(rec[m[4]:m[4] + m[3]], tpu) for m in meta if m[0] == kind]
        rows = [r for r in rows if r["rays"] > 0]
        if not rows:
            continue
        D = np.array([r["D"] for r in rows])
        out[KIND.get(kind, str(kind))] = {
            "launches": len(rows),
            "time_us": float(D.sum()),
            "mean_launch_us": float(D.mean()),
            "wave_live_frac": float(sum(r["life_frac"] * r["D"] for r in rows) / D.sum()),
            "below25_frac": float(sum(r["below25"] for r in rows) / D.sum()),
            "dry_frac": float(sum(r["dry"] for r in rows) / D.sum()),
            "rays_per_launch": float(np.mean([r["rays"] for r in rows])),
            "by_bounce": {},
        }
        for b in sorted(set(meta[meta[:, 0] == kind][:, 2].tolist())):
            rb = [launch_stats(rec[m[4]:m[4] + m[3]], tpu) for m in meta if m[0] == kind and m[2] == b]
            rb = [r for r in rb if r["rays"] > 0]
            if rb:
                Db = np.array([r["D"] for r in rb])
                out[KIND.get(kind, str(kind))]["by_bounce"][int(b)] = {
                    "launches": len(rb), "mean_launch_us": round(float(Db.mean()), 1),
                    "rays_per_launch": round(float(np.mean([r["rays"] for r in rb]))),
                    "below25_frac": round(float(sum(r["below25"] for r in rb) / Db.sum()), 3),
                    "dry_frac": round(float(sum(r["dry"] for r in rb) / Db.sum()), 3),
                    "working_waves": round(float(np.mean([r["working_waves"] for r in rb]))),
                    "wave_life_us_p50_p90_max": [round(float(np.mean([r[k] for r in rb])), 1)
                                                 for k in ("life_p50", "life_p90", "life_max")]}
    return out


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
    import wpt_loader

    pkg = wpt_loader.load()
    itf = pkg.interface
    cloud = pkg.scenes.triangle_cloud(100000)
    W, H = 1920, 1080
    itf.init(W, H, 2, *pkg.scenes.scene_camera(2))
    itf.store_mesh(1, cloud)
    if cfg == "c5":
        itf.update_settings(2, 2, 1, 1, 0)
        itf.set_render_options(8, 0xBABABEBE, 0)
        n = W * H * 1024
    elif cfg == "c3":
        itf.update_settings(1, 1, 0, 0, 0)
        itf.set_render_options(8, 0xBABABEBE, 1 << 27)
        n = W * H * 64
    else:  # the reference's init defaults (RR only)
        itf.set_render_options(0, 0xBABABEBE, 0)
        n = W * H * 16
    # optional launch options: argv[3] = "name=value,name=value"
    for kv in (sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] else []):
        k, v = kv.split("=")
        itf.set_option(k, v)
    itf.compute(n)  # warm-up: photons, first rounds, buffers
    itf.sync()
    # the probed call starts from an empty sample stock, as bench.py's timed one
    itf.set_option("stock", itf.get_option("stock"))
    itf.sync()
    itf.set_option("probe", cap)
    t0 = time.perf_counter()
    itf.compute(n)
    itf.sync()
    wall = time.perf_counter() - t0
    meta, rec, tpu = itf.probe_read()
    itf.set_option("probe", 0)
    grid_pct, trace_pct = itf.get_option("grid_pct"), itf.get_option("trace_grid_pct")
    itf.shutdown()
    # resident capacity of the traversal kernels (waves), from the probed
    # grids: the fused k_trace's grid is trace_grid_pct of it, the separate
    # kernels' multi-lane grids grid_pct
    tr = meta[meta[:, 0] == 5]
    cap = (int(tr[:, 3].max()) * 100 // trace_pct if len(tr) else
           int(meta[:, 3].max()) * 100 // grid_pct if len(meta) else 1)
    res = {"config": cfg, "options": sys.argv[3] if len(sys.argv) > 3 else "", "compute_s": wall, "launches_recorded": int(len(meta)), "ticks_per_us": tpu,
           "note": "first launches of one compute call; times in microseconds",
           "gpu_wide": gpu_wide(meta, rec, tpu, cap) if len(meta) else None,
           "kernels": summarise(meta, rec, tpu)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Same-process A/B of launch options on the adaptive sessions of bench.py's
`secondary` block: C5 (PNEE + adaptive on both halves, depth 8, 1080p, one
compute of W*H*1024 after a warm-up compute of the same size) and the
reference's init defaults (left NormalNEE random, right PNEE adaptive,
RR-only, compute(W*H*16) x 3 after one warm-up call).

Fixed-spp sessions (c3, c2, museum: the bench's configs, compute(W*H*spp)
per call, `calls` calls after `warm_calls` warm-up calls) report a CRC of
the final frame's bits, which must agree across variants.

usage: python tools/session_rate.py c5|init|c3|c2|museum [--reps R] [--] "opt=v,opt=v" "opt=v" ...
Each variant (a comma-separated list of interface.OPTIONS settings, "" for
the defaults) runs R times, interleaved; one JSON line per run, then a
summary line with the median per variant."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import wpt_loader  # noqa: E402

SESSIONS = {
    "c5": dict(types=(2, 2), adaptive=(1, 1), depth=8, n=1920 * 1080 * 1024, calls=1, warm=1920 * 1080 * 1024),
    "init": dict(types=None, adaptive=None, depth=0, n=1920 * 1080 * 16, calls=3, warm=1920 * 1080 * 16),
    "c3": dict(types=(1, 1), adaptive=(0, 0), depth=8, n=1920 * 1080 * 64, calls=10, warm=1920 * 1080 * 64,
               warm_calls=2),
    "c2": dict(scene=101, types=(1, 1), adaptive=(0, 0), depth=4, n=1920 * 1080 * 64, calls=10, warm=1920 * 1080 * 64,
               warm_calls=2),
    "museum": dict(scene=0, types=(1, 1), adaptive=(0, 0), depth=8, n=1920 * 1080 * 64, calls=5,
                   warm=1920 * 1080 * 64, warm_calls=2),
}


def run(itf, pkg, cloud, name, opts, spp=0):
    c = dict(SESSIONS[name])
    if spp:  # a shorter budget per compute (profiling)
        c["n"] = c["warm"] = 1920 * 1080 * spp
    itf.set_option("defaults", 0)
    for o in opts:
        k, v = o.split("=", 1)
        itf.set_option(k, v)
    scene = c.get("scene", 2)
    itf.init(1920, 1080, scene, *pkg.scenes.scene_camera(scene))
    if scene == 2:
        itf.store_mesh(1, cloud)
    if c["types"]:
        itf.update_settings(c["types"][0], c["types"][1], c["adaptive"][0], c["adaptive"][1], 0)
    itf.set_render_options(c["depth"], 0xBABABEBE, 0)
    for _ in range(c.get("warm_calls", 1)):
        itf.compute(c["warm"])
    # the timed call starts from an empty sample stock (re-setting the option
    # drops the ring): every sample it adds was traced inside the window
    itf.set_option("stock", itf.get_option("stock"))
    itf.sync()
    itf.clear_stats()
    t0 = time.perf_counter()
    mark = lambda what: print(f"[mark {time.monotonic() * 1e3:.3f}] {what}", file=sys.stderr, flush=True)
    mark("window")
    for k in range(c["calls"]):
        itf.compute(c["n"])
        mark(f"call {k} returned")
    itf.sync()
    dt = time.perf_counter() - t0
    mark("end")
    st = itf.stats()
    crc = None
    if "warm_calls" in c:
        import zlib
        acc, cnt = itf.read_radiance(1920, 1080)
        crc = zlib.crc32(acc.tobytes()) ^ zlib.crc32(cnt.tobytes())
    itf.shutdown()
    return {"session": name, "crc": crc, "ms_per_call": round(dt * 1e3 / c["calls"], 3), "options": opts, "s": round(dt, 4), "Mray/s": (st["rays"] + st["shadow_rays"]) / dt / 1e6,
            "rays": st["rays"] + st["shadow_rays"], "paths": st["paths"],
            **{k: st[k] for k in ("stock_traced", "stock_consumed", "stock_deficit", "stock_waits", "plan_us", "stock_us",
                                  "fill_paths", "stock_rays", "finish_paths", "finish_max_bounces", "bounces")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session", choices=sorted(SESSIONS))
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--spp", type=int, default=0, help="budget per compute in W*H units (default: the bench's)")
    ap.add_argument("variants", nargs="*", default=[""])
    a = ap.parse_intermixed_args()
    pkg = wpt_loader.load()
    itf = pkg.interface
    itf.set_device(0)
    cloud = pkg.scenes.triangle_cloud(100000)
    res = {}
    for _ in range(a.reps):
        for v in a.variants:
            opts = [o for o in v.split(",") if o]
            r = run(itf, pkg, cloud, a.session, opts, a.spp)
            print(json.dumps(r), flush=True)
            res.setdefault(v, []).append(r["Mray/s"])
    print(json.dumps({"summary": {v: {"median": statistics.median(x), "all": [round(y, 1) for y in x]}
                                  for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()

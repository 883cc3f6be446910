"""Throughput of a session left at the reference's init defaults (left half
NormalNEE + random sampling, right half PNEE + adaptive, wasm_interface.rs:
90-94) on the C3 scene at 1080p: compute(n) in chunks of W*H*16 paths after
one warm-up chunk. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import wpt_loader  # noqa: E402

pkg = wpt_loader.load()
itf = pkg.interface
W, H = 1920, 1080
itf.set_device(0)
opts = [a for a in sys.argv[2:] if "=" in a]  # launch options NAME=VALUE (interface.OPTIONS)
for o in opts:
    k, v = o.split("=", 1)
    itf.set_option(k, v)
itf.init(W, H, 2, *pkg.scenes.scene_camera(2))
itf.store_mesh(1, pkg.scenes.triangle_cloud(100000))
itf.compute(W * H * 16)
itf.sync()
itf.clear_stats()
chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 4
t0 = time.perf_counter()
for _ in range(chunks):
    itf.compute(W * H * 16)
itf.sync()
dt = time.perf_counter() - t0
st = itf.stats()
rays = st["rays"] + st["shadow_rays"]
print(json.dumps({"workload": "init defaults (left NormalNEE random, right PNEE adaptive), C3 scene 1080p",
                  "paths": chunks * W * H * 16, "s": dt, "Mray/s": rays / dt / 1e6,
                  "finish_paths": st["finish_paths"],
                  "finish_max_bounces": st["finish_max_bounces"],
                  "lib": os.environ.get("WPT_LIB_VARIANT", "product"), "options": opts}))
itf.shutdown()

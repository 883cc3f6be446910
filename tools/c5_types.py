"""C5-shaped adaptive session (bunny scene, 1080p, depth 8, both halves
adaptive, 1024 spp budget) with a chosen render type per half, to price the
PNEE light pick against uniform NEE: one warm-up step, one timed step, kernel
busy times. Usage: tools/c5_types.py <left_type> <right_type> [NAME=VALUE ...]"""
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
lt, rt = int(sys.argv[1]), int(sys.argv[2])
for o in sys.argv[3:]:
    k, v = o.split("=", 1)
    itf.set_option(k, v)
itf.set_device(0)
itf.init(W, H, 2, *pkg.scenes.scene_camera(2))
itf.store_mesh(1, pkg.scenes.triangle_cloud(100000))
itf.update_settings(lt, rt, 1, 1, 0)
itf.set_render_options(8, 0xBABABEBE, 0)
n = W * H * 1024
itf.compute(n)
itf.sync()
itf.clear_stats()
itf.set_profiling(True)
t0 = time.perf_counter()
itf.compute(n)
itf.sync()
dt = time.perf_counter() - t0
st = itf.stats()
kt = itf.kernel_times()
print(json.dumps({"types": [lt, rt], "Mray/s": (st["rays"] + st["shadow_rays"]) / dt / 1e6, "s": dt,
                  "busy_ms": {k: round(v["busy_ms"], 1) for k, v in kt.items()}}))
itf.shutdown()

"""Run the C3 workload once with counting on in a WPT_STAMPS build and print
the extend kernel's per-wave cycle split (tools/exp builds only)."""
import os
import sys

import torch  # noqa: F401

sys.path.insert(0, ".")
import wpt_loader  # noqa: E402

w = wpt_loader.load()
itf = w.interface
W, H, spp = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 8
itf.init(W, H, 2, *w.scenes.scene_camera(2))
itf.store_mesh(1, w.scenes.triangle_cloud(100000))
itf.update_settings(1, 1, 0, 0, 0)
itf.set_render_options(8, 0xBABABEBE, 1 << 27)
itf.set_counting(True)
itf.compute(W * H * spp)
itf.sync()
st = itf.stats()
keys = ["stamp_expand", "stamp_leaf", "stamp_pop", "stamp_refill", "stamp_loop"]
tot = st["stamp_loop"]
print({k: round(st[k] / tot, 3) for k in keys})
it = st["ext_lane_iters"] / 64
print("cycles per wave-iteration:", {k: round(st[k] / it, 1) for k in keys})
print("steps/ray", st["ext_live_iters"] / st["rays"], "live", st["ext_live_iters"] / st["ext_lane_iters"])

"""Robustness runs on the GPU: a 1M-triangle mesh (scene load incl. the GPU BVH build,
closest-hit parity on a ray sample against the oracle) and a 4K frame."""
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, ".")
sys.path.insert(0, "oracle")
import pyoracle  # noqa: E402
import wpt_loader  # noqa: E402

w = wpt_loader.load()
itf = w.interface
cloud = w.scenes.triangle_cloud(1_000_000)
t0 = time.time()
itf.init(3840, 2160, 2, *w.scenes.scene_camera(2))
itf.store_mesh(1, cloud)
print("1M-triangle scene build + upload", round(time.time() - t0, 2), "s, BVH depth", itf.bvh_depth(), "BVH2 build (ms, on GPU)", itf.scene_build_info(), flush=True)
rng = np.random.default_rng(3)
n = 20000
o = (np.array([-0.9, 5.4, 0.4], np.float32) + rng.uniform(-0.5, 0.5, (n, 3))).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
d[:, 1] = -np.abs(d[:, 1])
d[:, 2] = np.abs(d[:, 2])
d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
rays = np.concatenate([o, d], axis=1).astype(np.float32)
tg, ig = itf.trace_rays(rays)
t0 = time.time()
tr, ir, _ = pyoracle.OracleScene(2, cloud).trace_rays(rays)
print("oracle 1M build+trace", round(time.time() - t0, 1), "s", flush=True)
print("1M closest hit bit-exact:", bool(np.array_equal(ig, ir) and np.array_equal(tg.view(np.uint32), tr.view(np.uint32))),
      flush=True)
itf.update_settings(1, 1, 0, 0, 0)
itf.set_render_options(8, 0xBABABEBE, 0)
t0 = time.time()
itf.compute(3840 * 2160 * 4)
itf.sync()
st = itf.stats()
dt = time.time() - t0
print("4K x 4 spp on the 1M mesh:", round(dt, 2), "s,", round((st["rays"] + st["shadow_rays"]) / dt / 1e6), "Mray/s",
      flush=True)
acc, cnt = itf.read_radiance(3840, 2160)
print("all pixels sampled 4x:", bool(np.all(cnt == 4)), "finite:", bool(np.isfinite(acc).all()), flush=True)

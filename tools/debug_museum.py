"""GPU smoke of the museum scene (torus): extend / shadow parity hooks on
random rays, then a tiny render; prints progress after each step."""
import sys
import time

import numpy as np
import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import wpt_loader  # noqa: E402

w = wpt_loader.load()
itf = w.interface
step = sys.argv[1] if len(sys.argv) > 1 else "all"
itf.init(32, 24, 0, *w.scenes.scene_camera(0))
print("scene ok", flush=True)
rng = np.random.default_rng(5)
n = 20000
o = rng.uniform([-18.0, -0.9, -18.0], [18.0, 2.5, 18.0], (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
rays = np.concatenate([o, d], axis=1).astype(np.float32)
if step in ("all", "ext"):
    for k in (1, 10, 100, 1000, 20000):
        t0 = time.time()
        t, i = itf.trace_rays(rays[:k])
        print("extend", k, "ok", round(time.time() - t0, 3), flush=True)
if step in ("all", "shadow"):
    lights = np.arange(1, 109, dtype=np.int32)  # after the plane: lights come early? use debug scene
    ds = itf.DebugScene(0)
    li = ds.lights().astype(np.int32)
    sh = ds.shapes()
    for k in (1, 10, 100, 1000, 20000):
        L = li[rng.integers(0, len(li), k)]
        q = sh[L, :3]
        pq = np.concatenate([rays[:k, :3], q], axis=1).astype(np.float32)
        t0 = time.time()
        occ = itf.shadow_rays(pq, L)
        print("shadow", k, "ok", round(time.time() - t0, 3), occ.mean(), flush=True)
itf.update_settings(1, 1, 0, 0, 0)
itf.set_render_options(4, 0xBABABEBE, 0)
for k in (1, 64, 32 * 24):
    itf.compute(k)
    print("render", k, "ok", flush=True)

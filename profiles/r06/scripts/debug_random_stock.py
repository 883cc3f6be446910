"""Debug: one random + one adaptive half with the random half's rounds from
the stock (WPT_OPT_STOCK_RANDOM) against the same session without it and the
oracle's; prints where the frame, counts or sampling view differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
import wpt_loader  # noqa: E402

W, H, DEPTH = 48, 32, 4
CHUNKS = (1500, 4000, 6100, 9000)
pkg = wpt_loader.load()
itf = pkg.interface
itf.set_device(0)
mesh = pkg.scenes.triangle_cloud(3000, seed=0x5EED)
cam = pkg.scenes.scene_camera(2)
types, adaptive = (1, 1), (0, 1)
for batch in (900, 0):
    out = {}
    for sr in (0, 1):
        itf.set_option("defaults", 0)
        itf.set_option("stock_random", sr)
        itf.init(W, H, 2, *cam)
        itf.store_mesh(1, mesh)
        itf.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
        itf.set_render_options(DEPTH, 0xBABABEBE, batch)
        res = []
        for n in CHUNKS:
            itf.compute(n)
            acc, cnt = itf.read_radiance(W, H)
            res.append((acc.copy(), cnt.copy(), itf.results(1, W, H).copy()))
        out[sr] = res
        itf.shutdown()
    ref = pyoracle.OracleScene(2, mesh).adaptive(W, H, cam, types, adaptive, DEPTH)
    for i, n in enumerate(CHUNKS):
        ref.compute(n)
        ra, rc, rs = ref.read()
        for sr in (0, 1):
            a, c, s = out[sr][i]
            da = np.argwhere(np.any(a.view(np.uint32) != ra.view(np.uint32), axis=-1))
            dc = np.argwhere(c != rc)
            ds = np.argwhere(np.any(s != rs, axis=-1))
            print(f"batch {batch} call {i} sr {sr}: acc diff {len(da)} cnt diff {len(dc)} samp diff {len(ds)}"
                  f" cols acc {sorted(set(da[:, 1].tolist()))[:12]} cnt {sorted(set(dc[:, 1].tolist()))[:12]}"
                  f" samp {sorted(set(ds[:, 1].tolist()))[:12]}", flush=True)

"""Diagnostic: closest hits of random rays in the museum scene (scene 0)
through the product's trace_rays hook and the oracle; reports rays whose
results differ. Usage: WPT_LIB_VARIANT=<v> python tools/torus_ghosts.py N"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import wpt_loader  # noqa: E402
import pyoracle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
pkg = wpt_loader.load()
itf = pkg.interface
cam = pkg.scenes.scene_camera(0)
itf.set_device(0)
itf.init(64, 64, 0, *cam)
rng = np.random.default_rng(5)
o = np.stack([rng.uniform(-20, 20, n), rng.uniform(-1, 2, n), rng.uniform(-12, 12, n)], 1)
d = rng.normal(size=(n, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.concatenate([o, d], 1).astype(np.float32)
t_g, id_g = itf.trace_rays(rays)
itf.shutdown()
t_r, id_r, _ = pyoracle.OracleScene(0, None).trace_rays(rays)
bad = np.nonzero((id_g != id_r) | (t_g.view(np.uint32) != t_r.view(np.uint32)))[0]
out = {"lib": os.environ.get("WPT_LIB_VARIANT", ""), "rays": n, "mismatches": int(bad.size),
       "examples": [{"ray": rays[i].tolist(), "gpu": [float(t_g[i]), int(id_g[i])], "oracle": [float(t_r[i]), int(id_r[i])]}
                    for i in bad[:8]]}
print(json.dumps(out))

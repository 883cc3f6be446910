"""BVH2 build time, host (wpt_scene.cpp) vs GPU (wpt_bvh_gpu.hip), on
triangle clouds of growing size; the two trees are checked equal. Prints one
JSON object (profiles/r02/bvh_build_times.json)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import wpt_loader  # noqa: E402

wpt = wpt_loader.load()
itf = wpt.interface
rows = []
for n in (int(a) for a in (sys.argv[1:] or ["10000", "100000", "1000000", "4000000"])):
    mesh = wpt.scenes.triangle_cloud(n, seed=77)
    g = itf.DebugScene(2, mesh, gpu=True)  # first: the GPU builder's buffers are allocated here
    g = itf.DebugScene(2, mesh, gpu=True)
    h = itf.DebugScene(2, mesh)
    same = bool(np.array_equal(h.nodes()[:, 6:], g.nodes()[:, 6:]) and
                np.array_equal(h.shapes().view(np.uint32), g.shapes().view(np.uint32)))
    rows.append({"triangles": n, "nodes": h.num_nodes, "depth": h.depth, "host_ms": round(h.bvh_ms, 2),
                 "gpu_ms": round(g.bvh_ms, 2), "speedup": round(h.bvh_ms / g.bvh_ms, 1), "same_tree": same})
    print(rows[-1], file=sys.stderr, flush=True)
print(json.dumps({"what": "BVH2 build (bvh.rs:103-437): host wall clock vs GPU device time incl. its H2D/D2H copies; "
                          "scene = display_obj over a triangle cloud", "rows": rows}))

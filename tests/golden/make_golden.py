"""Generate tests/golden/golden.npz: small outputs of the oracle (the CPU
restatement of the reference, oracle/) that regression-pin both the oracle
and the HIP path. The reference itself cannot be built here (Rust/WASM, no
toolchain: DESIGN.md §3), so these vectors are oracle outputs, not reference
outputs; the oracle is pinned to the reference's definitions by
tests/test_oracle_kat.py.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (scene id, width, height, spp, max depth, left type, right type)
IMAGES = [
    (100, 32, 32, 2, 1, 0, 1),   # C1 box, NoNEE | NEE halves
    (101, 40, 24, 2, 4, 1, 1),   # C2 spheres, BVH disabled
    (2, 40, 24, 2, 8, 1, 1),     # C3 scene with a 3000-triangle cloud
    (2, 24, 16, 2, 0, 1, 0),     # unbounded RR loop
]
SEED = 0xBABABEBE
CLOUD = dict(n=3000, seed=0x5EED)


def rays_for(scene_id, n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform([-2.0, -0.9, -1.0], [2.0, 5.5, 9.0], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    return np.concatenate([o, d], axis=1).astype(np.float32)


def main():
    import pyoracle
    import wpt_loader
    scenes = wpt_loader.load().scenes
    cloud = scenes.triangle_cloud(CLOUD["n"], seed=CLOUD["seed"])
    out = {"cloud_params": np.array([CLOUD["n"], CLOUD["seed"]], np.int64), "seed": np.array([SEED], np.uint32)}
    for i, (sid, w, h, spp, depth, lt, rt) in enumerate(IMAGES):
        sc = pyoracle.OracleScene(sid, cloud if sid == 2 else None)
        cam = scenes.scene_camera(sid)
        acc, _ = sc.render(w, h, cam, lt, rt, depth, SEED, 0, spp, threads=4)
        out[f"img{i}_cfg"] = np.array([sid, w, h, spp, depth, lt, rt], np.int64)
        out[f"img{i}_acc"] = acc
    for sid in (2, 100, 101):
        sc = pyoracle.OracleScene(sid, cloud if sid == 2 else None)
        rays = rays_for(sid, 2000, 1000 + sid)
        t, ids, _ = sc.trace_rays(rays)
        out[f"hits{sid}_rays"] = rays
        out[f"hits{sid}_t"] = t
        out[f"hits{sid}_id"] = ids
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz"), **out)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()

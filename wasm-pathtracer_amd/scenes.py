"""Scene inputs that the reference builds on its JavaScript side.

* ``triangle_cloud`` mirrors ``triangleCloud(n)`` (src_ts/client/index.ts:165-184):
  centres U[-2.5,2.5]² × U[0,5], each vertex = centre + U[0,0.5]³, stored as
  f32 (``Float32Array``). ``Math.random`` is replaced by a seeded splitmix64
  stream (53-bit doubles in [0,1)) so the mesh is reproducible; the reference
  loads it into mesh slot 1 in place of the missing ``bunny2.obj``
  (SURVEY §0 F2).
* ``scene_camera`` mirrors ``sceneCamera`` (index.ts:153-162).
* ``parse_obj`` mirrors ``parseObj`` (src_ts/client/obj_parser.ts:3-51) and the
  bunny transform of index.ts:213-221 (×(8, 8, -8)).
"""
import numpy as np

MASK64 = (1 << 64) - 1


def _splitmix64(seed):
    state = seed & MASK64
    while True:
        state = (state + 0x9E3779B97F4A7C15) & MASK64
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        z ^= z >> 31
        yield (z >> 11) * (1.0 / (1 << 53))


def triangle_cloud(n, seed=0x5EED):
    """index.ts:165-184 with a seeded PRNG. Returns float32 array (9*n,)."""
    rnd = _splitmix64(seed)
    out = np.empty(9 * n, dtype=np.float64)
    for i in range(n):
        cx = next(rnd) * 5 - 2.5
        cy = next(rnd) * 5 - 2.5
        cz = next(rnd) * 5
        for k in range(3):
            out[9 * i + 3 * k + 0] = cx + next(rnd) * 0.5
            out[9 * i + 3 * k + 1] = cy + next(rnd) * 0.5
            out[9 * i + 3 * k + 2] = cz + next(rnd) * 0.5
    return out.astype(np.float32)


def scene_camera(scene_id):
    """index.ts:153-162 → (x, y, z, rot_x, rot_y). Build-defined configs
    (SURVEY §8d): 100 = C1 box, 101 = C2 spheres (bunny camera)."""
    if scene_id == 0:
        return (0.0, 16.34, -23.76, 0.54, 0.0)
    if scene_id in (1, 2, 101):
        return (-0.9, 5.4, 0.4, 0.58, 0.0)
    if scene_id == 100:
        return (0.0, 1.0, -3.5, 0.0, 0.0)
    raise ValueError("No Scene")


def parse_obj(text, bunny_transform=True):
    """obj_parser.ts:3-51 (split on single spaces, 'v' and triangular 'f'
    only) followed by index.ts:216-220's ×(8, 8, -8) for the bunny."""
    verts = []
    faces = []
    for line in text.split("\n"):
        segs = line.split(" ")
        if segs[0] == "v":
            verts.append((float(segs[1]), float(segs[2]), float(segs[3])))
        elif segs[0] == "f":
            if len(segs) != 4:
                raise ValueError("Non-triangular face in OBJ file")
            faces.extend(int(s.split("/")[0]) - 1 for s in segs[1:4])
    v = np.asarray(verts, dtype=np.float32)
    out = v[np.asarray(faces, dtype=np.int64)].reshape(-1).astype(np.float32)
    if bunny_transform:
        out = out.reshape(-1, 3)
        out[:, 0] *= np.float32(8)
        out[:, 1] *= np.float32(8)
        out[:, 2] *= np.float32(-8)
        out = out.reshape(-1)
    return out

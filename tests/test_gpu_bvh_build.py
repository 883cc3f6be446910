"""GPU BVH2 build (wpt_bvh_gpu.hip) against the host build (wpt_scene.cpp,
bvh.rs:103-437; itself pinned to the oracle by test_host_scene_matches_oracle).

The same scene built both ways must give the same tree: node boxes equal as
f32 values (a bound of ±0 may carry the other sign: min / max of +0 and -0 is
order-dependent on the host and no box test can tell them apart), node
ranges / child indices, the reordered shapes, the light list, the depth and
the BVH4 collapsed from it all bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same_scene(itf, scene_id, mesh):
    h = itf.DebugScene(scene_id, mesh)
    g = itf.DebugScene(scene_id, mesh, gpu=True)
    assert g.bvh_on_gpu and not h.bvh_on_gpu
    assert (g.num_shapes, g.num_inf, g.num_nodes, g.num_lights, g.depth, g.use_bvh, g.tri_only) == \
           (h.num_shapes, h.num_inf, h.num_nodes, h.num_lights, h.depth, h.use_bvh, h.tri_only)
    hn, gn = h.nodes(), g.nodes()
    assert np.array_equal(hn[:, 6:], gn[:, 6:])                       # left_first, count
    assert np.array_equal(hn[:, :6].view(np.float32), gn[:, :6].view(np.float32), equal_nan=True)  # boxes (== on f32)
    assert np.array_equal(h.shapes().view(np.uint32), g.shapes().view(np.uint32))
    assert np.array_equal(h.lights(), g.lights())
    h4, g4 = h.nodes4(), g.nodes4()
    assert h4.shape == g4.shape
    assert np.array_equal(h4[:, 24:], g4[:, 24:])
    assert np.array_equal(h4[:, :24].view(np.float32), g4[:, :24].view(np.float32), equal_nan=True)
    return h, g


@pytest.mark.parametrize("n", [1, 2, 3, 7, 100, 3000, 100000])
def test_cloud(wpt, n):
    _same_scene(wpt.interface, 2, wpt.scenes.triangle_cloud(n, seed=0xC10D + n))


@pytest.mark.parametrize("scene_id", [0, 100, 101])
def test_builtin_scenes(wpt, scene_id):
    """museum (tori, AA rects, 108 lights), the C1 box, C2's spheres."""
    _same_scene(wpt.interface, scene_id, None)


def test_degenerate_inputs(wpt):
    """Equal centroids (nothing to bin: one leaf), centroids on a line, exact
    and negative zeros (the bunny transform's z * -8 of z = 0)."""
    itf = wpt.interface
    tri = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], np.float32)
    _same_scene(itf, 2, np.tile(tri, 500))
    line = np.concatenate([tri + np.float32(i) * np.array([1, 0, 0] * 3, np.float32) for i in range(300)])
    _same_scene(itf, 2, line)
    rng = np.random.default_rng(5)
    v = rng.integers(-3, 4, size=(2000, 3, 3)).astype(np.float32)
    v[..., 2] *= np.float32(-8)                   # zeros become -0.0
    _same_scene(itf, 2, v.reshape(-1))


@pytest.mark.parametrize("n", [3000, 70000])
def test_nan_triangles(wpt, n):
    """Triangles with NaN vertices (wpt_parse_obj emits them for face indices
    out of range, as obj_parser.ts reads `undefined`): f32::min / max skip a
    NaN (bvh.rs:412-424, aabb.rs:90-100), so the GPU build must skip it too
    and give the host's tree; 70000 shapes are also what a session builds on
    the GPU by default."""
    itf = wpt.interface
    v = wpt.scenes.triangle_cloud(n, seed=0xBAD).reshape(-1, 3, 3).copy()
    rng = np.random.default_rng(3)
    idx = rng.choice(n, size=n // 20, replace=False)
    v[idx[: len(idx) // 2]] = np.nan                      # whole triangles
    v[idx[len(idx) // 2:], rng.integers(0, 3), :] = np.nan  # one vertex each
    v[idx[:5], :, 0] = -np.float32(np.nan)               # negative NaN bits
    _same_scene(itf, 2, v.reshape(-1))


def test_million_triangles(wpt):
    h, g = _same_scene(wpt.interface, 2, wpt.scenes.triangle_cloud(1_000_000, seed=77))
    print(f"BVH2 build of 1M triangles: host {h.bvh_ms:.1f} ms, GPU {g.bvh_ms:.1f} ms")


def test_session_builds_large_meshes_on_gpu(wpt, cloud_small):
    """wpt_init / store_mesh: >= 65536 finite shapes -> GPU build; smaller -> host."""
    session = wpt.interface
    cam = wpt.scenes.scene_camera(2)
    session.set_device(0)
    session.init(32, 32, 2, *cam)
    try:
        session.store_mesh(1, cloud_small)
        assert session.scene_build_info()[1] is False
        session.store_mesh(1, wpt.scenes.triangle_cloud(70000, seed=3))
        ms, on_gpu = session.scene_build_info()
        assert on_gpu and ms > 0
    finally:
        session.shutdown()


def test_obj_ingestion_renders_like_store_mesh(wpt):
    """wpt_load_obj + wpt_notify_mesh_loaded (the OBJ route into mesh slot 1)
    gives the frame of the same vertices handed over by mesh_vertices."""
    itf = wpt.interface
    mesh = wpt.scenes.triangle_cloud(2000, seed=21)
    v = mesh.reshape(-1, 3)
    doc = "".join(f"v {float(a)!r} {float(b)!r} {float(c)!r}\n" for a, b, c in v.tolist())
    doc += "".join(f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}\n" for i in range(len(v) // 3))
    cam = wpt.scenes.scene_camera(2)
    frames = []
    for route in ("store", "obj"):
        itf.set_device(0)
        itf.init(48, 32, 2, *cam)
        try:
            if route == "store":
                itf.store_mesh(1, mesh)
            else:
                assert itf.load_obj(1, doc) == len(v)
                assert itf.notify_mesh_loaded(1)
            itf.update_settings(1, 1, 0, 0, 0)
            itf.set_render_options(4, 0xBABABEBE, 0)
            itf.compute(48 * 32 * 8)
            frames.append(itf.read_radiance(48, 32)[0])
        finally:
            itf.shutdown()
    assert np.array_equal(frames[0].view(np.uint32), frames[1].view(np.uint32))
    assert frames[0].max() > 0

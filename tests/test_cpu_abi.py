"""CPU-only checks of the product's host side: the C ABI library loads and
exports every symbol include/wpt.h declares, the host scene/BVH build is
bit-identical to the oracle's restatement of bvh.rs/scene.rs, and calls that
need a session fail with the reference's error (not a crash)."""
import ctypes

import numpy as np
import pytest


def test_library_exports_header(wpt):
    L = wpt.lib()
    declared = wpt._lib.header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    # every declared symbol has a ctypes signature in the binding
    assert sorted(wpt._lib.EXPORTED) == declared


def test_reference_exports_are_mirrored(wpt):
    """The 12 #[wasm_bindgen] exports of wasm_interface.rs have a wpt_ twin
    and a same-named Python mirror."""
    ref_exports = ["init", "results", "update_scene", "update_settings", "update_viewport", "update_camera",
                   "allocate_mesh", "mesh_vertices", "notify_mesh_loaded", "allocate_texture",
                   "notify_texture_loaded", "compute"]
    L = wpt.lib()
    for name in ref_exports:
        assert hasattr(L, "wpt_" + name)
        assert callable(getattr(wpt.interface, name))


def test_calls_without_session_fail_cleanly(wpt):
    itf = wpt.interface
    for fn, args in [(itf.compute, (10,)), (itf.update_scene, (2,)), (itf.update_camera, (0, 0, 0, 0, 0)),
                     (itf.update_viewport, (8, 8)), (itf.allocate_mesh, (1, 3)), (itf.stats, ())]:
        with pytest.raises(itf.WptError) as e:
            fn(*args)
        assert e.value.code == itf.ERR_NOT_INIT
    assert not wpt.lib().wpt_results(0)
    assert wpt.lib().wpt_last_error() == b"init not called"


@pytest.mark.parametrize("scene_id", [0, 2, 100, 101])
def test_host_scene_matches_oracle(wpt, oracle, cloud_small, scene_id):
    """Product BVH2 build (wpt_scene.cpp) == oracle restatement of bvh.rs:
    identical nodes (bounds bits, left_first, count), shape order, lights."""
    mesh = cloud_small if scene_id == 2 else None
    d = wpt.interface.DebugScene(scene_id, mesh)
    o = oracle.OracleScene(scene_id, mesh)
    assert (d.num_shapes, d.num_inf, d.num_nodes, d.num_lights) == (o.num_shapes, o.num_inf, o.num_nodes, o.num_lights)
    assert np.array_equal(d.nodes(), o.nodes())
    assert np.array_equal(d.shapes().view(np.uint32), o.shapes().view(np.uint32))
    assert d.use_bvh == (o.bvh_kind == 2)
    assert o.verify_bvh()


def test_host_scene_100k_matches_oracle(wpt, oracle, cloud_100k):
    d = wpt.interface.DebugScene(2, cloud_100k)
    o = oracle.OracleScene(2, cloud_100k)
    assert np.array_equal(d.nodes(), o.nodes())
    assert np.array_equal(d.shapes().view(np.uint32), o.shapes().view(np.uint32))
    assert o.verify_bvh()
    assert 10 < d.depth < 64


def test_scene_catalogue(wpt):
    with pytest.raises(wpt.interface.WptError):
        wpt.interface.DebugScene(7)
    m = wpt.interface.DebugScene(0)  # museum (scenes.rs:15-55): plane, 27 tori, 108 light triangles, 10 boxes
    assert (m.num_shapes, m.num_inf, m.num_lights) == (146, 1, 108)
    s = wpt.interface.DebugScene(2)  # display_obj without a mesh: 2 planes + 2 light triangles
    assert (s.num_shapes, s.num_inf, s.num_lights) == (4, 2, 2)
    assert list(s.lights()) == [2, 3]
    s = wpt.interface.DebugScene(101)
    assert s.use_bvh == 0 and s.num_shapes == 20


def test_triangle_cloud_shape(wpt):
    c = wpt.scenes.triangle_cloud(1000, seed=1)
    assert c.dtype == np.float32 and c.shape == (9000,)
    v = c.reshape(-1, 3, 3)
    ctr = v.min(axis=1)
    assert ctr[:, 0].min() >= -2.5 and ctr[:, 0].max() <= 3.0
    assert ctr[:, 2].min() >= 0.0 and ctr[:, 2].max() <= 5.5
    assert np.all(v.max(axis=1) - v.min(axis=1) <= 0.5)
    assert np.array_equal(c, wpt.scenes.triangle_cloud(1000, seed=1))


def test_parse_obj(wpt):
    txt = "# c\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1\n"
    v = wpt.scenes.parse_obj(txt)
    assert np.array_equal(v, np.array([0, 0, -0.0, 8, 0, -0.0, 0, 8, -0.0], np.float32))
    with pytest.raises(ValueError):
        wpt.scenes.parse_obj("v 0 0 0\nf 1 1 1 1\n")


@pytest.mark.parametrize("scene_id,n", [(2, 100000), (2, 3000), (2, 7), (2, 1), (0, 0), (100, 0)])
def test_bvh4_collapse_matches_oracle(wpt, oracle, scene_id, n):
    """The BVH4 is bvh4.rs's DP tree cut (r_cost / collapse_with, :127-281)
    with the F4 leaf-encoding fix: the product build and the oracle's
    restatement give the same nodes, children, leaf ranges and boxes bit for
    bit; every finite shape sits in exactly one leaf and every child box lies
    inside its node's hull (BVHNode4::verify, bvh4.rs:300-376)."""
    mesh = wpt.scenes.triangle_cloud(n, seed=0x5EED) if n else None
    ref = oracle.OracleScene(scene_id, mesh).bvh4()
    d = wpt.interface.DebugScene(scene_id, mesh)
    got = d.nodes4()
    assert np.array_equal(got, ref)
    assert 1 <= got.shape[0] <= max(1, d.num_nodes // 2)
    covered = np.zeros(d.num_shapes - d.num_inf, np.int32)
    for row in got:
        k = int(row[0])
        assert 1 <= k <= 4 and np.all(row[1 + 9 * k:] == 0)
        slots = row[1: 1 + 9 * k].reshape(k, 9)
        for s in slots:
            if s[0] == 2:
                covered[s[1]: s[1] + s[2]] += 1
            else:
                assert s[0] == 1
                child = got[s[1]]
                cb = child[1: 1 + 9 * int(child[0])].reshape(-1, 9)[:, 3:].view(np.float32)
                box = s[3:].view(np.float32)
                assert np.all(cb[:, :3] >= box[:3]) and np.all(cb[:, 3:] <= box[3:])
    assert np.all(covered == 1)


def _f32(hexbits):
    return np.frombuffer(bytes.fromhex(hexbits), "<f4")[0]


def test_obj_parser_number_semantics(wpt):
    """wpt_parse_obj (obj_parser.ts:3-51 in libwpt.so) against parseFloat /
    parseInt / Float32Array as node evaluates them (tests/golden/
    obj_numbers.json, made by tests/golden/make_obj_golden.js)."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "obj_numbers.json")))
    fl = [e for e in g["floats"] if " " not in e["s"] and "\n" not in e["s"]]
    doc = "".join(f"v {e['s']} 0 0\n" for e in fl) + "".join(f"f {i + 1} {i + 1} {i + 1}\n" for i in range(len(fl)))
    got = wpt.interface.parse_obj(doc).reshape(-1, 9)[:, 0]
    for e, x in zip(fl, got):
        want = _f32(e["f32"])
        assert (np.isnan(want) and np.isnan(x)) or want.view(np.uint32) == x.view(np.uint32), e["s"]
    ints = [e for e in g["ints"] if " " not in e["s"] and "\n" not in e["s"]]
    nv = 120
    doc = "".join(f"v {k} 0 0\n" for k in range(nv)) + "".join(f"f {e['s']} 1 1\n" for e in ints)
    got = wpt.interface.parse_obj(doc).reshape(-1, 9)[:, 0]
    for e, x in zip(ints, got):
        idx = np.frombuffer(bytes.fromhex(e["f64"]), "<f8")[0] - 1.0
        want = idx if (idx == idx and 0 <= idx < nv) else np.nan
        assert (np.isnan(want) and np.isnan(x)) or float(x) == want, e["s"]


def test_obj_parser_matches_restatement(wpt):
    """A generated OBJ (vertices, normals, comments, 'f a//n' and 'f a/t/n'
    corners, CRLF line ends) through libwpt.so and through the Python
    restatement (scenes.parse_obj), both with index.ts's (8, 8, -8) scale."""
    rng = np.random.default_rng(11)
    v = rng.normal(size=(300, 3)).astype(np.float32)
    f = rng.integers(1, 301, size=(500, 3))
    lines = ["# generated", "o mesh"] + [f"v {a!r} {b!r} {c!r}" for a, b, c in v.tolist()] + ["vn 0 1 0"]
    lines += [f"f {a}//1 {b}/2/1 {c}" + ("\r" if k % 3 == 0 else "") for k, (a, b, c) in enumerate(f.tolist())]
    doc = "\n".join(lines) + "\n"
    got = wpt.interface.parse_obj(doc, scale=(8, 8, -8))
    want = wpt.scenes.parse_obj(doc)
    assert got.shape == (500 * 9,)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    with pytest.raises(wpt.interface.WptError):
        wpt.interface.parse_obj("v 0 0 0\nf 1 1 1 1\n")
    assert wpt.interface.parse_obj("").size == 0


def test_bvh4_large_leaves(wpt, oracle):
    """Stacks of coincident triangles give BVH2 leaves of 200, 70 and 40
    shapes; the BVH4 child code keeps an inline leaf's count in 6 bits, so
    the leaves of >= 64 go through the leaf table (an inline count of 64-127
    would set the leaf-table flag bit)."""
    tri = np.array([-0.5, 0.2, 5.5, 0.6, 0.4, 5.8, 0.0, 1.3, 5.6], np.float32)
    stacks = [np.tile(tri + np.float32(dx) * np.array([1, 0, 0] * 3, np.float32), k)
              for dx, k in ((0.0, 200), (1.2, 70), (-1.3, 40))]
    mesh = np.concatenate([wpt.scenes.triangle_cloud(500, seed=3)] + stacks)
    d = wpt.interface.DebugScene(2, mesh)
    assert not d.bvh_on_gpu and d.bvh_ms >= 0.0
    leaf_counts = sorted(int(c) for c in d.nodes()[:, 7] if c >= 40)
    assert leaf_counts == [40, 70, 200]
    got = d.nodes4()
    assert np.array_equal(got, oracle.OracleScene(2, mesh).bvh4())
    counts4 = sorted(int(s[2]) for row in got for s in row[1: 1 + 9 * int(row[0])].reshape(-1, 9) if s[0] == 2)
    assert [c for c in counts4 if c >= 40] == [40, 70, 200]


def test_comm_entry_points(wpt):
    """The RCCL communicator of the C ABI (wpt_comm_unique_id, wpt_set_comm,
    wpt_gather_frame, wpt_comm_destroy): a 128-byte id without a GPU, clean
    errors without a session."""
    itf = wpt.interface
    uid = itf.comm_unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128
    assert wpt.lib().wpt_comm_unique_id(None) == itf.ERR_INVALID_ARG
    for fn, args in [(itf.set_comm, (0, 2, 16, uid)), (itf.gather_frame, (0,)), (itf.comm_destroy, ())]:
        with pytest.raises(itf.WptError) as e:
            fn(*args)
        assert e.value.code == itf.ERR_NOT_INIT


def test_launch_option_ranges(wpt):
    """Session-less launch options (defaults of the next init): traversal
    0 / 1 / 3 accepted, 2 (the removed fast tree) and the removed fast-tree
    options 15-19 and 21 rejected; the probe option accepted."""
    L = wpt.lib()
    itf = wpt.interface
    try:
        for v in (0, 1, 3):
            assert L.wpt_set_option(1, v) == 0 and L.wpt_set_option(2, v) == 0
        assert L.wpt_set_option(1, 2) == itf.ERR_INVALID_ARG
        assert L.wpt_set_option(2, 4) == itf.ERR_INVALID_ARG
        for opt in (15, 16, 17, 18, 19, 21):
            assert L.wpt_set_option(opt, 1) == itf.ERR_INVALID_ARG
        assert L.wpt_set_option(22, 0) == 0
    finally:
        L.wpt_set_option(1, 3)
        L.wpt_set_option(2, 3)

"""GPU parity: libwpt.so's HIP kernels against the oracle (CPU restatement of
the reference) on identical inputs and identical per-path RNG seeds.

Bar (north_star): image relative L2 <= 1e-4 against the CPU reference; in
practice the kernels restate the reference's f32 op order exactly, so hits
and images are expected to be bit-identical and the tests also report the
bit-exact fraction.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4  # north_star: "within 1e-4 relative L2"


@pytest.fixture(params=["bvh4", "bvh2"])
def session(wpt, request):
    """Every test runs twice: the BVH4 fast path (with the exact re-trace of
    flagged rays) and the exact BVH2 stack machine alone (wpt_set_option
    WPT_OPT_TRAVERSAL and _SH, set for every session the test starts). The
    default, auto, is one of the two per scene."""
    itf = wpt.interface
    itf.set_option("traversal", request.param)
    itf.set_option("traversal_sh", request.param)
    yield itf
    try:
        itf.shutdown()
    except itf.WptError:
        pass
    itf.set_option("defaults", 0)


def _start(itf, wpt, scene_id, w, h, mesh=None, max_depth=0, seed=0xBABABEBE, types=(1, 1)):
    cam = wpt.scenes.scene_camera(scene_id)
    itf.init(w, h, scene_id, *cam)
    if mesh is not None:
        assert itf.store_mesh(1, mesh) == (scene_id == 2)
    itf.update_settings(types[0], types[1], 0, 0, 0)
    itf.set_render_options(max_depth, seed, 0)
    return cam


def _random_rays(rng, n, scene_id):
    """Rays from the camera region and from inside the scene, random dirs."""
    o = np.empty((n, 3), np.float32)
    half = n // 2
    cam = [0.0, 16.34, -23.76] if scene_id == 0 else [-0.9, 5.4, 0.4]
    o[:half] = np.array(cam, np.float32) + rng.uniform(-0.5, 0.5, (half, 3)).astype(np.float32)
    if scene_id == 0:  # museum: tori at y = -0.5, walls up to y = 2
        lo, hi = [-18.0, -0.9, -18.0], [18.0, 2.5, 18.0]
    elif scene_id == 100:
        lo, hi = [-1.9, -0.9, -1.0], [1.9, 2.9, 3.9]
    else:
        lo, hi = [-2.0, -0.9, 3.0], [2.0, 3.0, 9.0]
    o[half:] = rng.uniform(lo, hi, (n - half, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    # camera-half rays look roughly down/forward, as primary rays do
    d[:half, 1] = -np.abs(d[:half, 1])
    d[:half, 2] = np.abs(d[:half, 2])
    # a few axis-aligned directions (inv_dir = inf in the slab test)
    d[half: half + 8] = np.eye(3, dtype=np.float32)[np.arange(8) % 3] * np.where(np.arange(8) % 2, 1, -1)[:, None]
    return np.concatenate([o, d], axis=1).astype(np.float32)


@pytest.mark.parametrize("scene_id", [0, 2, 100, 101])
def test_closest_hit_bit_exact(wpt, oracle, session, cloud_small, scene_id):
    """Scene::trace_g (scene.rs:162-184): (t, shape id) bitwise equal."""
    mesh = cloud_small if scene_id == 2 else None
    _start(session, wpt, scene_id, 64, 64, mesh)
    ref = oracle.OracleScene(scene_id, mesh)
    rays = _random_rays(np.random.default_rng(1234 + scene_id), 20000, scene_id)
    t_g, id_g = session.trace_rays(rays)
    t_r, id_r, _ = ref.trace_rays(rays)
    assert np.array_equal(id_g, id_r), f"{np.sum(id_g != id_r)} id mismatches"
    assert np.array_equal(t_g.view(np.uint32), t_r.view(np.uint32))
    assert (id_g >= 0).mean() > 0.3


def test_closest_hit_100k(wpt, oracle, session, cloud_100k):
    _start(session, wpt, 2, 64, 64, cloud_100k)
    ref = oracle.OracleScene(2, cloud_100k)
    rays = _random_rays(np.random.default_rng(99), 50000, 2)
    t_g, id_g = session.trace_rays(rays)
    t_r, id_r, _ = ref.trace_rays(rays)
    assert np.array_equal(id_g, id_r), f"{np.sum(id_g != id_r)} id mismatches"
    assert np.array_equal(t_g.view(np.uint32), t_r.view(np.uint32))


def test_closest_hit_large_leaves(wpt, oracle, session, cloud_small):
    """Leaves of many primitives: stacks of coincident triangles cannot be
    split (bvh.rs:423-424), so the BVH2 keeps leaves of 200, 70 and 40 shapes;
    in the BVH4 a leaf of >= 64 shapes goes through the leaf table (child
    codes keep the count in 6 bits). Exact ties between the copies resolve in
    the reference's order."""
    tri = np.array([-0.5, 0.2, 5.5, 0.6, 0.4, 5.8, 0.0, 1.3, 5.6], np.float32)
    stacks = [np.tile(tri + np.float32(dx) * np.array([1, 0, 0] * 3, np.float32), k)
              for dx, k in ((0.0, 200), (1.2, 70), (-1.3, 40))]
    mesh = np.concatenate([cloud_small] + stacks)
    _start(session, wpt, 2, 64, 64, mesh)
    ref = oracle.OracleScene(2, mesh)
    rays = _random_rays(np.random.default_rng(4321), 20000, 2)
    t_g, id_g = session.trace_rays(rays)
    t_r, id_r, _ = ref.trace_rays(rays)
    assert np.array_equal(id_g, id_r), f"{np.sum(id_g != id_r)} id mismatches"
    assert np.array_equal(t_g.view(np.uint32), t_r.view(np.uint32))
    counts = wpt.interface.DebugScene(2, mesh).nodes()[:, 7]
    assert counts.max() >= 64


@pytest.mark.parametrize("scene_id", [0, 2, 100, 101])
def test_shadow_query_exact(wpt, oracle, session, cloud_small, scene_id):
    """Scene::shadow_ray (scene.rs:104-133) incl. the early-exit shortcut."""
    mesh = cloud_small if scene_id == 2 else None
    _start(session, wpt, scene_id, 64, 64, mesh)
    ref = oracle.OracleScene(scene_id, mesh)
    rng = np.random.default_rng(7 + scene_id)
    n = 20000
    shapes = ref.shapes()
    lights = np.nonzero(shapes[:, 13] == 1.0)[0].astype(np.int32)
    li = lights[rng.integers(0, len(lights), n)]
    v = shapes[li, :9].reshape(n, 3, 3)
    a, b = rng.random((n, 1), dtype=np.float32), rng.random((n, 1), dtype=np.float32)
    sa = np.sqrt(a)
    q = (1 - sa) * v[:, 0] + sa * (1 - b) * v[:, 1] + sa * b * v[:, 2]
    rays = _random_rays(rng, n, scene_id)
    p = rays[:, :3]
    pq = np.concatenate([p, q.astype(np.float32)], axis=1)
    occ_g = session.shadow_rays(pq, li)
    occ_r = ref.shadow_rays(pq, li)
    assert np.array_equal(occ_g, occ_r), f"{np.sum(occ_g != occ_r)} mismatches"
    assert 0.01 < occ_g.mean() < 0.99


def _rel_l2(a, b):
    return float(np.linalg.norm((a - b).ravel().astype(np.float64)) / max(np.linalg.norm(b.ravel().astype(np.float64)), 1e-30))


@pytest.mark.parametrize("scene_id,max_depth,types", [
    (2, 8, (1, 1)), (2, 0, (1, 0)), (100, 1, (0, 1)), (100, 4, (1, 1)), (101, 4, (1, 1)), (101, 0, (0, 0)),
    (0, 4, (1, 1)), (0, 0, (0, 1)),
])
def test_image_parity(wpt, oracle, session, cloud_small, scene_id, max_depth, types):
    """Whole path loop (tracer.rs:224-330): radiance sums per pixel."""
    W, H, spp = 48, 32, 4
    mesh = cloud_small if scene_id == 2 else None
    cam = _start(session, wpt, scene_id, W, H, mesh, max_depth=max_depth, types=types)
    session.compute(W * H * spp)
    acc_g, cnt_g = session.read_radiance(W, H)
    ref = oracle.OracleScene(scene_id, mesh)
    acc_r, _ = ref.render(W, H, cam, types[0], types[1], max_depth, 0xBABABEBE, 0, spp, threads=4)
    assert np.all(cnt_g == spp)
    exact = np.mean(np.all(acc_g.view(np.uint32) == acc_r.view(np.uint32), axis=2))
    l2 = _rel_l2(acc_g, acc_r)
    print(f"scene {scene_id} depth {max_depth}: bit-exact pixels {exact:.6f}, rel L2 {l2:.3e}")
    assert l2 <= REL_L2_TOL
    assert exact == 1.0


@pytest.mark.parametrize("scene_id,max_depth,types", [(2, 0, (1, 2)), (2, 5, (2, 1)), (2, 3, (0, 1)), (0, 2, (1, 2)),
                                                     (100, 0, (1, 1))])
def test_image_parity_light_debug(wpt, oracle, session, cloud_small, scene_id, max_depth, types):
    """The reference's light-debug view: update_settings(.., is_light_debug=1)
    sets is_debug_photons (wasm_interface.rs:198-199), which changes the
    emitter rule (only paths that have not bounced add an emitter,
    tracer.rs:246-249) and replaces the shadow ray by an unconditional
    throughput * intensity for a light sample facing the hit (:297-299).
    NEE and PNEE halves (light pick from the photon octree), RR-only and
    capped paths; NoNEE halves ignore the flag except for the emitter rule."""
    W, H, spp = 48, 32, 4
    mesh = cloud_small if scene_id == 2 else None
    cam = wpt.scenes.scene_camera(scene_id)
    session.init(W, H, scene_id, *cam)
    if mesh is not None:
        session.store_mesh(1, mesh)
    session.update_settings(types[0], types[1], 0, 0, 1)
    session.set_render_options(max_depth, 0xBABABEBE, 0)
    session.compute(W * H * spp)
    acc_g, cnt_g = session.read_radiance(W, H)
    st = session.stats()
    ref = oracle.OracleScene(scene_id, mesh)
    acc_r, rst = ref.render(W, H, cam, types[0], types[1], max_depth, 0xBABABEBE, 0, spp, threads=4, light_debug=1)
    assert np.all(cnt_g == spp)
    assert st["shadow_rays"] == 0 and rst["shadow_rays"] == 0  # no shadow ray in the debug view
    assert st["rays"] == rst["rays"]
    assert _rel_l2(acc_g, acc_r) <= REL_L2_TOL
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    # the view differs from the physically based render (NEE halves add light unconditionally)
    acc_n, _ = ref.render(W, H, cam, types[0], types[1], max_depth, 0xBABABEBE, 0, spp, threads=4)
    assert not np.array_equal(acc_n, acc_r)


def test_image_parity_100k_c3_like(wpt, oracle, session, cloud_100k):
    """C3's scene (100k-triangle stand-in for bunny2.obj), depth 8, NEE."""
    W, H, spp = 64, 36, 2
    cam = _start(session, wpt, 2, W, H, cloud_100k, max_depth=8)
    session.compute(W * H * spp)
    acc_g, _ = session.read_radiance(W, H)
    acc_r, _ = oracle.OracleScene(2, cloud_100k).render(W, H, cam, 1, 1, 8, 0xBABABEBE, 0, spp, threads=8)
    assert _rel_l2(acc_g, acc_r) <= REL_L2_TOL
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))


def test_progressive_compute_matches_one_shot(wpt, session, cloud_small):
    """compute(n) calls accumulate in sample order: 3 calls == 1 call."""
    W, H = 40, 24
    _start(session, wpt, 2, W, H, cloud_small, max_depth=4)
    session.compute(W * H * 3)
    a1, c1 = session.read_radiance(W, H)
    session.set_render_options(4, 0xBABABEBE, 0)
    # each call gives the left half n/2 and the right half n - n/2 samples
    # (wasm_interface.rs:377-379): even n that cut both halves' rounds
    for n in (W * H - 6, W * H + 6, W * H):
        session.compute(n)
    a2, c2 = session.read_radiance(W, H)
    assert np.array_equal(c1, c2)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


def test_small_batches_match(wpt, session, cloud_small):
    """Batch size (paths resident per wavefront) does not change results."""
    W, H = 40, 24
    _start(session, wpt, 2, W, H, cloud_small, max_depth=0)
    session.compute(W * H * 3)
    a1, _ = session.read_radiance(W, H)
    session.set_render_options(0, 0xBABABEBE, 1000)
    session.compute(W * H * 3)
    a2, _ = session.read_radiance(W, H)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


def test_whole_round_pixel_order(wpt, session, cloud_small):
    """Batches of whole sample rounds trace the frame's pixels in tile order
    (WPT_OPT_PIXEL_TILE, default 8; 0 = raster): the (pixel, sample) pairs are the
    same, so the frame is the same bits for any tile size; a partial round
    keeps raster order. Ragged: 37x23 is no multiple of 8 or 5."""
    W, H = 37, 23
    frames = []
    # per half n/2 : n - n/2 (wasm_interface.rs:377-379): 851 px, halves of
    # 18 x 23 = 414 and 19 x 23 = 437 px; 828 = 2 rounds of the left half,
    # 874 = 2 of the right: whole rounds of each half (tiled batches), then
    # partial rounds (raster order), then whole rounds again
    calls = (2 * 828, 828 + 874 + 1, 901, 2 * 874)
    for tile in (0, 8, 5, 4):
        _start(session, wpt, 2, W, H, cloud_small, max_depth=6)
        session.set_option("pixel_tile", tile)
        for n in calls:
            session.compute(n)
        acc, cnt = session.read_radiance(W, H)
        frames.append((acc, cnt))
        session.shutdown()
    for f, c in frames[1:]:
        assert np.array_equal(c, frames[0][1])
        assert np.array_equal(f.view(np.uint32), frames[0][0].view(np.uint32))
    assert int(frames[0][1][:, : W // 2].sum()) == sum(n // 2 for n in calls)


@pytest.mark.parametrize("W,H,calls", [(17, 5, (85, 3, 170, 41)), (3, 29, (87, 87, 1, 2)), (40, 24, (960, 1921))])
def test_random_halves_budget(wpt, oracle, session, cloud_small, W, H, calls):
    """Two random halves: compute(n) gives the left half n/2 and the right
    half n - n/2 samples (wasm_interface.rs:377-379, two RenderInstances),
    each half in its own sequence of rounds (one sample per pixel of the half
    per round). Odd widths split the halves unevenly; odd n give the right
    half the extra sample. Per-half counts and radiance bit for bit against
    the oracle's session in the same schedule."""
    cam = _start(session, wpt, 2, W, H, cloud_small, max_depth=4, types=(1, 0))
    for n in calls:
        session.compute(n)
    acc_g, cnt_g = session.read_radiance(W, H)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, (1, 0), (0, 0), 4)
    for n in calls:
        ref.compute(n)
    acc_r, cnt_r, _ = ref.read()
    assert int(cnt_g[:, : W // 2].sum()) == sum(n // 2 for n in calls)
    assert int(cnt_g[:, W // 2:].sum()) == sum(n - n // 2 for n in calls)
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_partitions_bitwise_identical(wpt, session, cloud_small, nranks):
    """Multi-GPU tile partition: the union of the partitions'
    radiance equals the single-GPU frame bitwise (ranks emulated in turn)."""
    W, H, spp = 50, 30, 2
    _start(session, wpt, 2, W, H, cloud_small, max_depth=8)
    session.compute(W * H * spp)
    full, _ = session.read_radiance(W, H)
    merged = np.zeros_like(full).reshape(-1, 3)
    seen = np.zeros(W * H, np.int32)
    for r in range(nranks):
        session.set_partition(r, nranks, 8)
        px = session.partition_pixels()
        session.compute(len(px) * spp)
        acc, cnt = session.read_radiance(W, H)
        merged[px] = acc.reshape(-1, 3)[px]
        seen[px] += 1
        assert np.all(cnt.reshape(-1)[px] == spp)
    assert np.all(seen == 1)
    assert np.array_equal(merged.reshape(full.shape).view(np.uint32), full.view(np.uint32))


def test_results_rgba_matches_render_target(wpt, oracle, session, cloud_small):
    """results() bytes = render_target.rs:62-64 quantisation of acc/cnt."""
    W, H, spp = 32, 20, 3
    _start(session, wpt, 2, W, H, cloud_small, max_depth=4)
    session.compute(W * H * spp)
    rgba = session.results(0, W, H)
    acc, cnt = session.read_radiance(W, H)
    v = acc / cnt[..., None].astype(np.float32)
    expect = (np.clip(np.minimum(v, np.float32(1.0)), 0, None) * np.float32(255.0)).astype(np.uint8)
    assert np.array_equal(rgba[..., :3], expect)
    assert np.all(rgba[..., 3] == 255)
    # sampling view after update_settings with two random halves: cleared to
    # black, nothing repaints it (wasm_interface.rs:185-201, sampling_strategy.rs:66-70)
    samp = session.results(1, W, H)
    assert np.all(samp[..., :3] == 0) and np.all(samp[..., 3] == 255)


@pytest.mark.parametrize("W,H", [(17, 5), (1, 1), (3, 29)])
def test_viewport_and_camera_updates_ragged(wpt, oracle, session, cloud_small, W, H):
    """update_viewport (wasm_interface.rs:219) and update_camera (:239) reset
    the accumulation; the next frame equals a fresh render at the new size and
    camera, including odd widths that split the NEE/no-NEE halves unevenly and
    a 1x1 viewport. compute(0) is a no-op."""
    spp, types = 3, (1, 0)
    _start(session, wpt, 2, 16, 16, cloud_small, max_depth=4, types=types)
    session.compute(16 * 16 * 2)
    session.update_viewport(W, H)
    cam = (-0.5, 5.0, 0.8, 0.5, 0.1)
    session.update_camera(*cam)
    session.compute(0)
    _, cnt0 = session.read_radiance(W, H)
    assert np.all(cnt0 == 0)
    # reset (wasm_interface.rs:137-150) clears the sampling view; random halves stay black
    samp = session.results(1, W, H)
    assert samp.shape == (H, W, 4) and np.all(samp[..., :3] == 0) and np.all(samp[..., 3] == 255)
    session.compute(W * H * spp)
    acc_g, cnt_g = session.read_radiance(W, H)
    # n/2 : n - n/2 per half (odd widths: unequal halves, wasm_interface.rs:377-379)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, types, (0, 0), 4)
    ref.compute(W * H * spp)
    acc_r, cnt_r, _ = ref.read()
    assert np.array_equal(cnt_g, cnt_r)
    assert int(cnt_g.sum()) == W * H * spp - (W * H * spp // 2 if W == 1 else 0)  # W = 1: the left half is empty
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    with pytest.raises(session.WptError) as e:
        session.update_viewport(0, 4)
    assert e.value.code == session.ERR_INVALID_ARG


def test_interface_errors(wpt, session):
    itf = session
    E = itf.WptError
    with pytest.raises(E) as e:
        itf.compute(10)
    assert e.value.code == itf.ERR_NOT_INIT
    itf.init(16, 16, 2, *wpt.scenes.scene_camera(2))
    with pytest.raises(E) as e:
        itf.init(16, 16, 2, 0, 0, 0, 0, 0)
    assert e.value.code == itf.ERR_ALREADY_INIT
    with pytest.raises(E) as e:
        itf.update_scene(7)
    assert e.value.code == itf.ERR_INVALID_SCENE
    with pytest.raises(E) as e:
        itf.update_settings(3, 1, 0, 0, 0)
    assert e.value.code == itf.ERR_INVALID_ARG
    with pytest.raises(E) as e:
        itf.mesh_vertices(9, 3)
    assert e.value.code == itf.ERR_NO_MESH
    assert itf.notify_texture_loaded(0) is False
    # scene 2 without a mesh: planes + light only (display_obj fallback)
    itf.compute(16 * 16)
    assert itf.stats()["paths"] == 256
    # mesh for another slot does not rebuild the scene
    assert itf.store_mesh(0, np.zeros(9, np.float32)) is False


def _preorder(child):
    order, stack = [], [0]
    while stack:
        n = stack.pop()
        order.append(n)
        if child[n]:
            stack.extend(range(int(child[n]) + 7, int(child[n]) - 1, -1))
    return np.array(order)


@pytest.mark.parametrize("scene_id", [0, 2, 100])
def test_photon_tree_matches_oracle(wpt, oracle, session, cloud_small, scene_id):
    """PNEE preprocessing (tracer.rs:126-152) + PhotonTree (photon_tree.rs):
    GPU-shot photons inserted on the host == oracle tree, node for node,
    CDFs bitwise, same number of photons shot."""
    mesh = cloud_small if scene_id == 2 else None
    _start(session, wpt, scene_id, 32, 32, mesh, types=(2, 2))
    ref = oracle.OracleScene(scene_id, mesh)
    child, cum, shot, stored = session.photon_tree(ref.num_lights)
    leafs_r, cum_r, shot_r, stored_r = ref.photon_tree(0xBABABEBE)
    assert (shot, stored) == (shot_r, stored_r)
    assert stored == 300000
    order = _preorder(child)
    assert len(order) == len(leafs_r)
    assert np.array_equal((child[order] == 0).astype(np.uint8), leafs_r)
    assert np.array_equal(cum[order].view(np.uint32), cum_r.view(np.uint32))


@pytest.mark.parametrize("scene_id,max_depth,types", [
    (2, 8, (2, 2)), (2, 0, (1, 2)), (100, 4, (2, 0)), (101, 4, (2, 2)), (0, 4, (2, 2)),
])
def test_image_parity_pnee(wpt, oracle, session, cloud_small, scene_id, max_depth, types):
    """PNEE light selection (tracer.rs:270-273, PhotonTree::sample)."""
    W, H, spp = 48, 32, 4
    mesh = cloud_small if scene_id == 2 else None
    cam = _start(session, wpt, scene_id, W, H, mesh, max_depth=max_depth, types=types)
    session.compute(W * H * spp)
    acc_g, _ = session.read_radiance(W, H)
    acc_r, _ = oracle.OracleScene(scene_id, mesh).render(W, H, cam, types[0], types[1], max_depth, 0xBABABEBE, 0,
                                                         spp, threads=8)
    exact = np.mean(np.all(acc_g.view(np.uint32) == acc_r.view(np.uint32), axis=2))
    l2 = _rel_l2(acc_g, acc_r)
    print(f"PNEE scene {scene_id}: bit-exact pixels {exact:.6f}, rel L2 {l2:.3e}")
    assert l2 <= REL_L2_TOL
    assert exact == 1.0
    assert session.stats()["photons"] == 300000


@pytest.mark.parametrize("scene_id,types,adaptive,batch", [
    (2, (1, 1), (0, 1), 0), (2, (1, 2), (1, 1), 777), (101, (0, 1), (1, 0), 0),
])
def test_adaptive_sampling_matches_oracle(wpt, oracle, session, cloud_small, scene_id, types, adaptive, batch):
    """AdaptiveSamplingStrategy (sampling_strategy.rs:77-230) in sample rounds:
    per-pixel sample counts, radiance and the sampling view (results(1)) equal
    the oracle's after compute() calls that cut rounds at arbitrary points."""
    W, H, depth = 40, 24, 4
    mesh = cloud_small if scene_id == 2 else None
    cam = wpt.scenes.scene_camera(scene_id)
    session.init(W, H, scene_id, *cam)
    if mesh is not None:
        session.store_mesh(1, mesh)
    session.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
    session.set_render_options(depth, 0xBABABEBE, batch)
    ref = oracle.OracleScene(scene_id, mesh).adaptive(W, H, cam, types, adaptive, depth)
    for n in (1000, 3000, 5000, 7000):
        session.compute(n)
        ref.compute(n)
    acc_g, cnt_g = session.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    assert np.array_equal(cnt_g, cnt_r)
    assert cnt_g.max() > 4  # adaptive rounds ran
    # each half gets its own budget, n/2 left and n - n/2 right (wasm_interface.rs:374-379)
    chunks = (1000, 3000, 5000, 7000)
    assert int(cnt_g[:, : W // 2].sum()) == sum(n // 2 for n in chunks)
    assert int(cnt_g[:, W // 2:].sum()) == sum(n - n // 2 for n in chunks)
    assert _rel_l2(acc_g, acc_r) <= REL_L2_TOL
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(session.results(1, W, H), samp_r)


def test_c5_settings_match_oracle(wpt, oracle, session, cloud_100k):
    """C5's own session (BASELINE configs[4]): both halves PNEE + adaptive
    sampling, depth 8, the 100k-triangle stand-in, on a 64x48 viewport, with
    compute() chunks that cut adaptive rounds at arbitrary points. Sample
    counts, radiance and the sampling view (results(1)) equal the oracle's
    session bit for bit (sampling_strategy.rs:122-219, photon_tree.rs:80-159,
    tracer.rs:103-152 / :270-278)."""
    W, H, depth = 64, 48, 8
    cam = wpt.scenes.scene_camera(2)
    session.init(W, H, 2, *cam)
    session.store_mesh(1, cloud_100k)
    session.update_settings(2, 2, 1, 1, 0)
    session.set_render_options(depth, 0xBABABEBE, 0)
    ref = oracle.OracleScene(2, cloud_100k).adaptive(W, H, cam, (2, 2), (1, 1), depth)
    chunks = (W * H * 6, W * H * 5 + 17, W * H * 9 + 5, 4099)
    for n in chunks:
        session.compute(n)
        ref.compute(n, threads=8)
    acc_g, cnt_g = session.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    assert np.array_equal(cnt_g, cnt_r)
    assert cnt_g.max() > 4  # adaptive rounds ran past the 4-sample start
    assert int(cnt_g[:, : W // 2].sum()) == sum(n // 2 for n in chunks)
    assert int(cnt_g[:, W // 2:].sum()) == sum(n - n // 2 for n in chunks)
    assert _rel_l2(acc_g, acc_r) <= REL_L2_TOL
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(session.results(1, W, H), samp_r)


def test_init_defaults_match_reference(wpt, oracle, session, cloud_small):
    """init without update_settings starts as the reference's UI does
    (wasm_interface.rs:90-94): left NormalNEE + random sampling, right PNEE +
    adaptive sampling, compute(n) split n/2 : n - n/2; the whole sampling
    view starts blue."""
    W, H = 40, 24
    cam = wpt.scenes.scene_camera(2)
    session.init(W, H, 2, *cam)
    samp0 = session.results(1, W, H)
    assert np.all(samp0[..., 2] == 255) and np.all(samp0[..., :2] == 0)
    # the mesh load rebuilds the scene (update_scene, wasm_interface.rs:154-169):
    # the view is cleared and only the adaptive half repaints itself blue
    session.store_mesh(1, cloud_small)
    samp1 = session.results(1, W, H)
    assert np.all(samp1[:, : W // 2, :3] == 0) and np.all(samp1[:, W // 2:, 2] == 255)
    chunks = (2000, 3000, 6000)
    for n in chunks:
        session.compute(n)
    acc_g, cnt_g = session.read_radiance(W, H)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, (1, 2), (0, 1), 0)
    for n in chunks:
        ref.compute(n)
    acc_r, cnt_r, samp_r = ref.read()
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert session.stats()["photons"] == 300000  # the right half renders PNEE
    assert np.array_equal(session.results(1, W, H), samp_r)


@pytest.mark.parametrize("adaptive", [False, True])
def test_lanes_bitwise_identical(wpt, session, cloud_small, adaptive):
    """A batch is cut into slices traced concurrently on 1-4 lanes (streams,
    WPT_OPT_LANES); the frame is the same bit for bit,
    in RR-only mode (lanes drained together) and in adaptive rounds."""
    W, H = 40, 24
    cam = wpt.scenes.scene_camera(2)
    out = []
    for lanes in (1, 2, 3, 4):
        session.set_option("lanes", lanes)
        session.set_device(0)
        session.init(W, H, 2, *cam)
        session.store_mesh(1, cloud_small)
        session.update_settings(1, 2 if adaptive else 0, int(adaptive), int(adaptive), 0)
        session.set_render_options(0, 0xBABABEBE, 0)
        for n in (W * H * 3 + 11, 5000, 2 * W * H - 3):
            session.compute(n)
        acc, cnt = session.read_radiance(W, H)
        out.append((acc, cnt, session.stats()["rays"]))
        session.shutdown()
    for acc, cnt, rays in out[1:]:
        assert np.array_equal(cnt, out[0][1])
        assert rays == out[0][2]
        assert np.array_equal(acc.view(np.uint32), out[0][0].view(np.uint32))


def test_set_lanes_mid_session(wpt, session, cloud_small):
    """wpt_set_lanes changes the lane count between compute calls (bench.py's
    serialised step); the frame is the same bit for bit, and counts outside
    1..8 (the streams a session makes) are refused; 8 lanes work too."""
    W, H = 64, 48
    cam = wpt.scenes.scene_camera(2)
    out = []
    for seq in ((4, 4, 4), (3, 1, 8)):
        session.set_device(0)
        session.init(W, H, 2, *cam)
        session.store_mesh(1, cloud_small)
        session.update_settings(1, 1, 0, 0, 0)
        session.set_render_options(0, 0xBABABEBE, 0)
        for lanes in seq:
            session.set_lanes(lanes)
            session.compute(W * H * 40 + 7)
        for bad in (0, 9):
            with pytest.raises(wpt.interface.WptError):
                session.set_lanes(bad)
        out.append(session.read_radiance(W, H))
        session.shutdown()
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))


def test_set_lanes_deeper_scene(wpt, session, cloud_small, cloud_100k):
    """lanes dropped to 1, a deeper scene loaded (100k triangles
    after 3k: a deeper BVH, hence more traversal-stack spill per lane), lanes
    raised to 4 again: every lane's spill area must have grown with the scene
    (size_grids sizes all lanes the session made). The frame equals a fresh
    4-lane session's on the deep scene, and no stack overflow is reported."""
    W, H = 64, 48
    cam = wpt.scenes.scene_camera(2)
    out = []
    for fresh in (False, True):
        session.set_device(0)
        session.init(W, H, 2, *cam)
        session.update_settings(1, 1, 0, 0, 0)
        if not fresh:
            session.store_mesh(1, cloud_small)
            session.set_lanes(1)
            session.compute(W * H * 4)
        session.store_mesh(1, cloud_100k)
        session.set_render_options(8, 0xBABABEBE, 0)  # reset: the frame restarts on the deep scene
        session.set_lanes(4)
        session.compute(W * H * 40 + 7)
        out.append(session.read_radiance(W, H))
        session.shutdown()
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))


@pytest.mark.parametrize("scene_id,max_depth,types", [(2, 0, (1, 1)), (2, 4, (1, 2)), (0, 3, (1, 0)), (101, 4, (1, 1))])
def test_fused_trace_matches_separate(wpt, session, cloud_small, scene_id, max_depth, types):
    """WPT_OPT_FUSED: bounce b's extension rays and bounce b-1's shadow rays traced
    by one kernel give the frame of the separate extend / shadow kernels bit
    for bit (RR-only mode, a depth cap, PNEE, and a scene without BVH)."""
    W, H = 40, 24
    cam = wpt.scenes.scene_camera(scene_id)
    mesh = cloud_small if scene_id == 2 else None
    out = []
    for fused in ("0", "1"):
        session.set_option("fused", int(fused))
        session.init(W, H, scene_id, *cam)
        if mesh is not None:
            session.store_mesh(1, mesh)
        session.update_settings(types[0], types[1], 0, 0, 0)
        session.set_render_options(max_depth, 0xBABABEBE, 0)
        session.compute(W * H * 3 + 7)
        acc, cnt = session.read_radiance(W, H)
        st = session.stats()
        out.append((acc, cnt, st["rays"], st["shadow_rays"]))
        session.shutdown()
    assert np.array_equal(out[0][1], out[1][1])
    assert out[0][2:] == out[1][2:]
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))


@pytest.mark.parametrize("scene_id,types,adaptive", [(2, (1, 1), (0, 0)), (2, (2, 0), (0, 1)), (0, (1, 0), (0, 0)),
                                                     (101, (1, 1), (0, 0))])
def test_finish_tail_matches_wavefront(wpt, oracle, session, cloud_small, scene_id, types, adaptive):
    """RR-only batches (no depth cap): once few paths are live, k_finish runs
    each remaining path to its end in one launch (trace, shade, shadow ray,
    RR per path) instead of one launch per bounce. The frame and the ray
    counts are the same as the all-wavefront run (WPT_OPT_FINISH_BELOW 0),
    whether the tail starts at bounce 4 (every path) or never; and against
    the oracle for random halves."""
    W, H = 48, 32
    mesh = cloud_small if scene_id == 2 else None
    cam = wpt.scenes.scene_camera(scene_id)
    chunks = (W * H * 3, W * H + 5)
    out = []
    for fb in (0, 1 << 30, 64):
        session.init(W, H, scene_id, *cam)
        if mesh is not None:
            session.store_mesh(1, mesh)
        session.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
        session.set_render_options(0, 0xBABABEBE, 0)
        session.set_option("finish_below", fb)
        for n in chunks:
            session.compute(n)
        acc, cnt = session.read_radiance(W, H)
        st = session.stats()
        out.append((acc, cnt, st["rays"], st["shadow_rays"]))
        # tail statistics: no handover with the threshold 0; with 2^30 every
        # path still live after bounce 4 goes to k_finish
        if fb == 0:
            assert st["finish_paths"] == 0 and st["finish_max_bounces"] == 0
        elif fb == 1 << 30 and scene_id != 101:
            assert st["finish_paths"] > 0 and st["finish_max_bounces"] >= 1
        session.shutdown()
    for acc, cnt, rays, sh in out[1:]:
        assert np.array_equal(cnt, out[0][1])
        assert (rays, sh) == out[0][2:]
        assert np.array_equal(acc.view(np.uint32), out[0][0].view(np.uint32))
    if adaptive == (0, 0):
        ref = oracle.OracleScene(scene_id, mesh).adaptive(W, H, cam, types, adaptive, 0)
        for n in chunks:
            ref.compute(n)
        acc_r, cnt_r, _ = ref.read()
        assert np.array_equal(cnt_r, out[0][1])
        assert np.array_equal(acc_r.view(np.uint32), out[0][0].view(np.uint32))

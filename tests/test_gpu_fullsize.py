"""Parity at the configs' full sizes (BASELINE.json configs).

The GPU renders the whole frame at the config's resolution, spp and depth;
the oracle (CPU restatement of tracer.rs:156-330 with the same per-path
seeds) renders the whole frame (C1) or bands of rows (C2, C3), which must
match bit for bit — and so within the north_star's 1e-4 relative L2.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0xBABABEBE


def _rel_l2(a, b):
    return float(np.linalg.norm((a - b).ravel().astype(np.float64)) /
                 max(np.linalg.norm(b.ravel().astype(np.float64)), 1e-30))


def _render_gpu(itf, wpt, scene_id, W, H, spp, depth, types, mesh=None):
    cam = wpt.scenes.scene_camera(scene_id)
    itf.init(W, H, scene_id, *cam)
    try:
        if mesh is not None:
            itf.store_mesh(1, mesh)
        itf.update_settings(types[0], types[1], 0, 0, 0)
        itf.set_render_options(depth, SEED, 0)
        itf.compute(W * H * spp)
        acc, cnt = itf.read_radiance(W, H)
    finally:
        itf.shutdown()
    assert np.all(cnt == spp)
    return cam, acc


@pytest.mark.parametrize("types", [(1, 1), (0, 1)])
def test_c1_full_frame(wpt, oracle, types):
    """C1: the Cornell box (scene 100), 256x256, 1 spp, depth 1, whole frame."""
    W, H, spp, depth = 256, 256, 1, 1
    cam, acc_g = _render_gpu(wpt.interface, wpt, 100, W, H, spp, depth, types)
    acc_r, _ = oracle.OracleScene(100).render(W, H, cam, types[0], types[1], depth, SEED, 0, spp, threads=8)
    assert _rel_l2(acc_g, acc_r) <= 1e-4
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert acc_g.max() > 0


def _bands(H):
    return [(0, 2), (H // 2 - 2, H // 2 + 2), (H - 2, H)]


def test_c2_full_size_row_bands(wpt, oracle):
    """C2: spheres + planes with the BVH disabled (scene 101), 1920x1080,
    64 spp, depth 4; the GPU's full frame against oracle row bands (top,
    middle, bottom)."""
    W, H, spp, depth = 1920, 1080, 64, 4
    cam, acc_g = _render_gpu(wpt.interface, wpt, 101, W, H, spp, depth, (1, 1))
    ref = oracle.OracleScene(101)
    for y0, y1 in _bands(H):
        acc_r, _ = ref.render(W, H, cam, 1, 1, depth, SEED, 0, spp, region=(0, y0, W, y1), threads=16)
        g, r = acc_g[y0:y1], acc_r[y0:y1]
        assert _rel_l2(g, r) <= 1e-4, (y0, y1)
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), (y0, y1)


def test_c3_full_size_row_bands(wpt, oracle, cloud_100k):
    """C3: the bunny scene over the 100k-triangle stand-in, 1920x1080,
    64 spp, depth 8, NormalNEE; the GPU's full frame against oracle row bands."""
    W, H, spp, depth = 1920, 1080, 64, 8
    cam, acc_g = _render_gpu(wpt.interface, wpt, 2, W, H, spp, depth, (1, 1), mesh=cloud_100k)
    ref = oracle.OracleScene(2, cloud_100k)
    for y0, y1 in _bands(H):
        acc_r, _ = ref.render(W, H, cam, 1, 1, depth, SEED, 0, spp, region=(0, y0, W, y1), threads=16)
        g, r = acc_g[y0:y1], acc_r[y0:y1]
        assert _rel_l2(g, r) <= 1e-4, (y0, y1)
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), (y0, y1)


def test_c4_tile_partitions_row_bands(wpt, oracle, cloud_100k):
    """C4 (BASELINE.json configs[3]): the bunny scene over the 100k stand-in at
    3840x2160, 256 spp, depth 8, NormalNEE, rendered as the 8-GPU job renders
    it: 16-px tiles dealt round-robin to 8 ranks (wpt_set_partition(r, 8, 16)),
    each rank's partition traced in turn on this GPU, the partitions merged
    into one frame. Checked bit for bit against oracle row bands at the top,
    middle and bottom, and a band straddling a tile-row border (rows 14-17:
    tile rows 0 and 1 belong to different rank sets)."""
    itf = wpt.interface
    W, H, spp, depth, nranks = 3840, 2160, 256, 8, 8
    cam = wpt.scenes.scene_camera(2)
    itf.init(W, H, 2, *cam)
    frame = np.zeros((H * W, 3), np.float32)
    owner = np.full(H * W, -1, np.int32)
    try:
        itf.store_mesh(1, cloud_100k)
        itf.update_settings(1, 1, 0, 0, 0)
        itf.set_render_options(depth, SEED, 0)
        for r in range(nranks):
            itf.set_partition(r, nranks, 16)
            pix = itf.partition_pixels()
            itf.compute(len(pix) * spp)
            acc, cnt = itf.read_radiance(W, H)
            assert np.all(cnt.ravel()[pix] == spp)
            assert np.all(owner[pix] == -1)  # every pixel belongs to one rank
            owner[pix] = r
            frame[pix] = acc.reshape(-1, 3)[pix]
        st = itf.stats()
    finally:
        itf.shutdown()
    assert np.all(owner >= 0)
    assert st["paths"] == W * H * spp
    frame = frame.reshape(H, W, 3)
    ref = oracle.OracleScene(2, cloud_100k)
    for y0, y1 in [(0, 2), (14, 18), (H // 2 - 1, H // 2 + 1), (H - 2, H)]:
        acc_r, _ = ref.render(W, H, cam, 1, 1, depth, SEED, 0, spp, region=(0, y0, W, y1), threads=16)
        g, rr = frame[y0:y1], acc_r[y0:y1]
        assert _rel_l2(g, rr) <= 1e-4, (y0, y1)
        assert np.array_equal(g.view(np.uint32), rr.view(np.uint32)), (y0, y1)
    assert frame.max() > 0

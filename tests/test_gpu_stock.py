"""The adaptive halves' sample stock (WPT_OPT_STOCK, wpt_stock.h): every
sample's path depends only on (pixel, sample index), and an adaptive round
only decides how many of its next samples each pixel takes
(sampling_strategy.rs:122-176), added in sample order (render_target.rs:55-65).
So refill batches on the async lanes trace each pixel's next samples into a
ring ahead of the rounds, and a round adds its samples from the ring, tracing
only the ones it lacks. Every test checks the frame bit for bit: against the
oracle's adaptive session (the reference's round structure restated), or
against the same session with the stock off; and a sample's rays count when a
round takes it, so the ray counts equal the no-stock session's call by call.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# every async option, so that each test states the settings it runs
BASE = {"stock": 256, "stock_lanes": 2, "stock_ahead": 6, "stock_extra": 2, "stock_every": 2, "fill": 0,
        "async_prio": 0, "async_grid_pct": 0, "async_oneshot": 0, "stock_prefill": 1, "async_fused_below": 0}


@pytest.fixture(params=["bvh2", "bvh4"])
def itf(wpt, request):
    i = wpt.interface
    i.set_option("traversal", request.param)
    i.set_option("traversal_sh", request.param)
    yield i
    try:
        i.shutdown()
    except i.WptError:
        pass
    i.set_option("defaults", 0)


def _session(itf, wpt, mesh, W, H, types, adaptive, depth, **opts):
    cam = wpt.scenes.scene_camera(2)
    for k, v in dict(BASE, **opts).items():
        itf.set_option(k, v)  # the defaults of the init below
    itf.init(W, H, 2, *cam)
    itf.store_mesh(1, mesh)
    if types is not None:
        itf.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
    itf.set_render_options(depth, 0xBABABEBE, 0)
    return cam


# chunks that cut rounds mid-way, one of them smaller than a half's pixels
CHUNKS = (40 * 24 * 5, 40 * 24 * 3 + 17, 211, 40 * 24 * 9 + 5, 4099)


@pytest.mark.parametrize("opts", [{}, {"stock_lanes": 1, "stock_every": 1}, {"stock_every": 3}, {"stock": 64, "stock_ahead": 1},
                                  {"async_oneshot": 1, "async_prio": 1}, {"stock_prefill": 0},
                                  {"stock": 1024, "stock_ahead": 24, "stock_extra": 8},
                                  {"stock": 1024, "stock_ahead": 40, "stock_extra": 8, "stock_every": 3},
                                  {"async_grid_pct": 100, "async_fused_below": 1 << 26}])
@pytest.mark.parametrize("depth,types,adaptive", [
    (8, (2, 2), (1, 1)),   # C5's settings: PNEE + adaptive on both halves, depth cap
    (0, (1, 2), (0, 1)),   # the reference's init defaults: RR-only, right adaptive
    (0, (2, 1), (1, 0)),   # mirrored: left adaptive
])
def test_stock_matches_oracle(wpt, oracle, itf, cloud_small, opts, depth, types, adaptive):
    W, H = 40, 24
    cam = _session(itf, wpt, cloud_small, W, H, types, adaptive, depth, **opts)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, types, adaptive, depth)
    for n in CHUNKS:
        itf.compute(n)
        ref.compute(n)
    acc_g, cnt_g = itf.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    st = itf.stats()
    assert cnt_g.max() > 8  # several adaptive rounds ran
    assert st["stock_consumed"] > 0 and st["stock_traced"] >= st["stock_consumed"]
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(itf.results(1, W, H), samp_r)


@pytest.mark.parametrize("depth", [8, 0])
def test_stock_on_off_identical_and_ray_counts(wpt, itf, cloud_small, depth):
    """The frame, counts and rays are the same with the stock on and off,
    after every call: a sample's rays count when a round takes it (each
    path's rays ride with its radiance into the ring), so both sessions count
    exactly the rays of the samples in the image."""
    W, H = 48, 32
    out = {}
    for stock in (0, 256):
        _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, stock=stock)
        per_call = []
        for n in (W * H * 7, W * H * 4 + 33, 977, W * H * 11):
            itf.compute(n)
            st = itf.stats()
            per_call.append((st["rays"], st["shadow_rays"], st["paths"]))
        acc, cnt = itf.read_radiance(W, H)
        out[stock] = (acc, cnt, per_call)
        itf.shutdown()
    (a0, c0, r0), (a1, c1, r1) = out[0], out[256]
    assert np.array_equal(c0, c1)
    assert np.array_equal(a0.view(np.uint32), a1.view(np.uint32))
    assert r0 == r1


def test_stock_dropped_on_reset(wpt, itf, cloud_small):
    """A reset (camera update, wasm_interface.rs:239-257) drops the ring and
    the refills in flight: the session after it equals a fresh session with
    the stock off."""
    W, H, depth = 40, 24, 8
    cam = _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth)
    itf.compute(W * H * 9 + 7)
    cam2 = list(cam)
    cam2[0] += 0.05
    itf.update_camera(*cam2)
    for n in (W * H * 6, 333):
        itf.compute(n)
    acc1, cnt1 = itf.read_radiance(W, H)
    itf.shutdown()
    _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, stock=0)
    itf.update_camera(*cam2)
    for n in (W * H * 6, 333):
        itf.compute(n)
    acc0, cnt0 = itf.read_radiance(W, H)
    assert np.array_equal(cnt0, cnt1)
    assert np.array_equal(acc0.view(np.uint32), acc1.view(np.uint32))


def test_stock_option_change_mid_session(wpt, itf, cloud_small):
    """Changing the ring size mid-session drops the stock (its samples are
    traced again later from the same seeds): the frame stays the same bits."""
    W, H, depth = 40, 24, 8
    chunks = (W * H * 6 + 17, W * H * 5 + 3, W * H * 2 + 101, W * H * 4)  # each cuts a round
    _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth)
    itf.compute(chunks[0])
    itf.set_option("stock", 64)  # a new ring (new memory)
    itf.compute(chunks[1])
    itf.set_option("stock", 64)  # the same size: the ring dropped, kept
    itf.compute(chunks[2])
    itf.set_option("stock", 0)
    itf.compute(chunks[3])
    acc1, cnt1 = itf.read_radiance(W, H)
    st = itf.stats()
    assert st["stock_traced"] >= st["stock_consumed"]
    itf.shutdown()
    _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, stock=0)
    for n in chunks:
        itf.compute(n)
    acc0, cnt0 = itf.read_radiance(W, H)
    assert np.array_equal(cnt0, cnt1)
    assert np.array_equal(acc0.view(np.uint32), acc1.view(np.uint32))


@pytest.mark.parametrize("types,adaptive", [((1, 2), (0, 1)), ((2, 1), (1, 0))])
def test_fill_matches_oracle(wpt, oracle, itf, cloud_small, types, adaptive):
    """One random and one adaptive half, RR-only (the reference's init
    defaults and their mirror): the random half's whole rounds outside its
    seam columns run on the fill lane beside the adaptive half's rounds
    (WPT_OPT_FILL). Budgets of whole rounds, of whole rounds plus a partial
    one, and below one round; an odd width (the halves differ). Counts,
    radiance and the sampling view equal the oracle's session bit for bit."""
    W, H = 41, 24
    cam = _session(itf, wpt, cloud_small, W, H, types, adaptive, 0, fill=1)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, types, adaptive, 0)
    nh = (W // 2) * H if types[0] == 1 else (W - W // 2) * H  # the random half's pixels
    n_whole = 2 * nh * 3  # three whole rounds for either half's share
    for n in (n_whole, n_whole + 2 * 37 + 1, 150, 2 * nh * 5 + 1):
        itf.compute(n)
        ref.compute(n)
    acc_g, cnt_g = itf.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    assert itf.stats()["fill_paths"] > 0  # whole random rounds ran on the fill lane
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(itf.results(1, W, H), samp_r)


@pytest.mark.parametrize("opts", [{}, {"async_prio": 1}, {"async_grid_pct": 30}, {"stock_lanes": 3},
                                  {"async_oneshot": 1, "async_prio": 1}, {"fill": 1}])
def test_async_options_bitwise(wpt, itf, cloud_small, opts):
    """The reference's init-default session under the async options: the
    same bits as with the async lanes off."""
    W, H = 40, 24
    out = []
    for o in ({"fill": 0, "stock": 0}, opts):
        _session(itf, wpt, cloud_small, W, H, None, None, 0, **o)
        for n in (W * H * 4, W * H * 3 + 9, 500):
            itf.compute(n)
        out.append(itf.read_radiance(W, H))
        itf.shutdown()
    (a0, c0), (a1, c1) = out
    assert np.array_equal(c0, c1)
    assert np.array_equal(a0.view(np.uint32), a1.view(np.uint32))

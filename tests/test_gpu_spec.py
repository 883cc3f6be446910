"""Speculated first samples of adaptive rounds (WPT_OPT_SPEC, Renderer::
issue_spec): while round r of an adaptive half runs, sample cnt_p of every
pixel of the half -- its first sample of round r + 1, which exists because
sampling_strategy.rs:162-163 gives every pixel ceil(1 + 32 * scaled) >= 1
samples per round -- is traced on the async lanes; round r + 1 adds it first
for that pixel. Every test checks the frame bit for bit: against the oracle's
adaptive session (the reference's round structure restated), or against the
same session with speculation off.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def _session(itf, wpt, mesh, W, H, types, adaptive, depth, spec=1, spec_lanes=1):
    cam = wpt.scenes.scene_camera(2)
    itf.set_option("spec", spec)
    itf.set_option("spec_lanes", spec_lanes)
    itf.init(W, H, 2, *cam)
    itf.store_mesh(1, mesh)
    itf.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
    itf.set_render_options(depth, 0xBABABEBE, 0)
    return cam


# chunks that cut rounds mid-way, one of them smaller than a half's pixels, so
# that a round's speculated samples are consumed over several compute calls
CHUNKS = (40 * 24 * 5, 40 * 24 * 3 + 17, 211, 40 * 24 * 9 + 5, 4099)


@pytest.mark.parametrize("spec_lanes", [1, 2])
@pytest.mark.parametrize("depth,types,adaptive", [
    (8, (2, 2), (1, 1)),   # C5's settings: PNEE + adaptive on both halves, depth cap
    (0, (1, 2), (0, 1)),   # the reference's init defaults: RR-only, right adaptive
    (0, (2, 1), (1, 0)),   # mirrored: left adaptive
])
def test_spec_matches_oracle(wpt, oracle, itf, cloud_small, spec_lanes, depth, types, adaptive):
    W, H = 40, 24
    cam = _session(itf, wpt, cloud_small, W, H, types, adaptive, depth, 1, spec_lanes)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, types, adaptive, depth)
    for n in CHUNKS:
        itf.compute(n)
        ref.compute(n)
    acc_g, cnt_g = itf.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    assert cnt_g.max() > 8  # several adaptive rounds ran
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(itf.results(1, W, H), samp_r)


@pytest.mark.parametrize("depth", [8, 0])
def test_spec_on_off_identical_and_ray_counts(wpt, itf, cloud_small, depth):
    """The frame and counts are the same bits with speculation on and off.
    Rays count when a speculated sample is consumed (its round completes), so
    the speculating session has counted at most the other's rays and at least
    those minus one speculated batch per half."""
    W, H = 48, 32
    out = {}
    for spec in (0, 1):
        _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, spec)
        per_call = []
        for n in (W * H * 7, W * H * 4 + 33, 977, W * H * 11):
            itf.compute(n)
            st = itf.stats()
            per_call.append(st["rays"] + st["shadow_rays"])
        acc, cnt = itf.read_radiance(W, H)
        out[spec] = (acc, cnt, per_call)
        itf.shutdown()
    (a0, c0, r0), (a1, c1, r1) = out[0], out[1]
    assert np.array_equal(c0, c1)
    assert np.array_equal(a0.view(np.uint32), a1.view(np.uint32))
    # one speculated batch = one sample of every pixel of a half: bounded by
    # the rays of W * H / 2 paths of the session's longest per-path average
    max_per_path = max(r0) / (c0.sum())
    for x0, x1 in zip(r0, r1):
        assert x1 <= x0
        assert x0 - x1 <= 2 * (W * H // 2) * max_per_path * 4


def test_spec_dropped_on_reset(wpt, itf, cloud_small):
    """A reset (camera update, wasm_interface.rs:239-257) drops the speculated
    samples of the old image: the session after it equals a fresh session
    with speculation off."""
    W, H, depth = 40, 24, 8
    cam = _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, 1)
    itf.compute(W * H * 9 + 7)
    cam2 = list(cam)
    cam2[0] += 0.05
    itf.update_camera(*cam2)
    for n in (W * H * 6, 333):
        itf.compute(n)
    acc1, cnt1 = itf.read_radiance(W, H)
    itf.shutdown()
    _session(itf, wpt, cloud_small, W, H, (2, 2), (1, 1), depth, 0)
    itf.update_camera(*cam2)
    for n in (W * H * 6, 333):
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
    cam = _session(itf, wpt, cloud_small, W, H, types, adaptive, 0, 1)
    ref = oracle.OracleScene(2, cloud_small).adaptive(W, H, cam, types, adaptive, 0)
    nh = (W // 2) * H if types[0] == 1 else (W - W // 2) * H  # the random half's pixels
    n_whole = 2 * nh * 3  # three whole rounds for either half's share
    for n in (n_whole, n_whole + 2 * 37 + 1, 150, 2 * nh * 5 + 1):
        itf.compute(n)
        ref.compute(n)
    acc_g, cnt_g = itf.read_radiance(W, H)
    acc_r, cnt_r, samp_r = ref.read()
    assert np.array_equal(cnt_g, cnt_r)
    assert np.array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    assert np.array_equal(itf.results(1, W, H), samp_r)


@pytest.mark.parametrize("opts", [{}, {"async_prio": 1}, {"async_grid_pct": 30}, {"spec_lanes": 2}])
def test_async_options_bitwise(wpt, itf, cloud_small, opts):
    """The init-default session under every async option: the same bits as
    with the async lanes off."""
    W, H = 40, 24
    out = []
    base = {"fill": 0, "spec": 0, "async_prio": 0, "async_grid_pct": 0, "spec_lanes": 1}
    for o in (base, dict(base, fill=1, spec=1, **opts)):
        for k, v in o.items():
            itf.set_option(k, v)  # the defaults of the next init
        cam = wpt.scenes.scene_camera(2)
        itf.init(W, H, 2, *cam)
        itf.store_mesh(1, cloud_small)
        for n in (W * H * 4, W * H * 3 + 9, 500):
            itf.compute(n)
        out.append(itf.read_radiance(W, H))
        itf.shutdown()
    (a0, c0), (a1, c1) = out
    assert np.array_equal(c0, c1)
    assert np.array_equal(a0.view(np.uint32), a1.view(np.uint32))

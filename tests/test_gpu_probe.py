"""The wave-timeline probe (WPT_OPT_PROBE, wpt_probe_read): a measurement
hook on the production traversal kernels. Its records must be consistent
(every ray a launch took is counted once, start <= dry <= end) and turning it
on must not change a single bit of the frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render(itf, wpt, cloud, probe, fused, adaptive=0):
    itf.init(96, 64, 2, *wpt.scenes.scene_camera(2))
    itf.store_mesh(1, cloud)
    if adaptive:
        # both halves NEE with adaptive rounds (PNEE would add photon rays,
        # traced in whole launches but counted only as far as they were used)
        itf.update_settings(1, 1, 1, 1, 0)
    else:
        itf.update_settings(1, 1, 0, 0, 0)
    itf.set_render_options(6, 0xBABABEBE, 0)
    itf.set_option("fused", fused)
    itf.set_option("probe", probe)
    itf.clear_stats()
    itf.compute(96 * 64 * (24 if adaptive else 3))
    itf.sync()
    acc, cnt = itf.read_radiance(96, 64)
    st = itf.stats()
    meta, rec, tpu = itf.probe_read()
    itf.shutdown()
    return acc, cnt, st, meta, rec, tpu


@pytest.mark.parametrize("fused,adaptive", [(0, 0), (1, 0), (0, 1)])
def test_probe_records_every_ray_and_changes_nothing(wpt, cloud_small, fused, adaptive):
    """...and the session's ray counts (stats) equal the rays the traversal
    launches took: adaptive rounds included, whose batches return before
    their counts are read (flush_counts)."""
    itf = wpt.interface
    try:
        acc0, cnt0, st0, meta0, _, _ = _render(itf, wpt, cloud_small, 0, fused, adaptive)
        acc1, cnt1, st1, meta, rec, tpu = _render(itf, wpt, cloud_small, 4096, fused, adaptive)
    finally:
        itf.set_option("defaults", 0)
    assert len(meta0) == 0
    assert np.array_equal(acc0.view(np.uint32), acc1.view(np.uint32)) and np.array_equal(cnt0, cnt1)
    assert len(meta) > 0 and tpu > 0
    assert set(meta[:, 0].tolist()) <= {1, 3, 5}
    if fused:
        assert 5 in set(meta[:, 0].tolist())
    taken = 0
    for kind, lane, bounce, waves, first in meta:
        r = rec[first:first + waves].astype(np.int64)
        t0 = r[:, 0].min()
        s, d, e = (r[:, 0] - t0) % (1 << 32), (r[:, 1] - t0) % (1 << 32), (r[:, 2] - t0) % (1 << 32)
        assert np.all(s <= d) and np.all(d <= e)
        taken += int(r[:, 3].sum())
    # every extension and shadow ray traced was taken by exactly one wave:
    # the rays counted when traced, and those traced into the adaptive
    # halves' sample stock (counted in rays only when a round takes them)
    traced = st1["rays"] + st1["shadow_rays"] - st1["stock_rays_used"] + st1["stock_rays"]
    assert taken == traced
    if adaptive:
        assert st1["stock_rays"] > 0 and st1["stock_rays_used"] > 0

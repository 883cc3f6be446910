"""The sample stock on a 4K viewport (3840x2160, PNEE + adaptive on both
halves, C5's settings): with compute(W*H*80) the first refills hold 311 M
samples, more than 8 batches of 2^25 paths, so their batches grow instead of
the call failing ("stock refill too large" before round 6's fix; the sizes
are in profiles/r06/refill_4k_log.txt). The frame and the sample counts must
be the same bits with the stock on and off."""
import zlib

import pytest

pytestmark = pytest.mark.gpu


def test_stock_4k_large_refills(wpt, cloud_100k):
    itf = wpt.interface
    W, H = 3840, 2160
    cam = wpt.scenes.scene_camera(2)
    out = []
    try:
        for stock in (1024, 0):
            itf.set_option("defaults", 0)
            itf.set_option("stock", stock)
            itf.init(W, H, 2, *cam)
            itf.store_mesh(1, cloud_100k)
            itf.update_settings(2, 2, 1, 1, 0)
            itf.set_render_options(8, 0xBABABEBE, 0)
            itf.compute(W * H * 80)
            st = itf.stats()
            acc, cnt = itf.read_radiance(W, H)
            out.append((zlib.crc32(acc.tobytes()), zlib.crc32(cnt.tobytes()), st["rays"], st["shadow_rays"],
                        st["stock_traced"]))
            itf.shutdown()
    finally:
        itf.set_option("defaults", 0)
    assert out[0][4] > 8 * (1 << 25)
    assert out[0][:4] == out[1][:4]

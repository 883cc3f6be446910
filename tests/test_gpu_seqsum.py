"""The adaptive rounds' mse_sum with its chunk effects computed on the GPU
(k_sum_chunks / k_sum_scan / k_sum_eff, as every round does) and walked in
order on the host: the sequential loop's bits on every input of
tests/test_seqsum.py."""
import ctypes

import numpy as np
import pytest

from test_seqsum import cases, same, seq, walk_cases

pytestmark = pytest.mark.gpu


def device(wpt, v):
    v = np.ascontiguousarray(v, np.float32)
    out = ctypes.c_float(0.0)
    rc = wpt.lib().wpt_seq_sum_device(v.ctypes.data_as(ctypes.c_void_p), len(v), ctypes.addressof(out))
    assert rc == 0, wpt.lib().wpt_last_error()
    return np.float32(out.value)


def test_device_chunk_sums_bit_exact(wpt):
    itf = wpt.interface
    itf.init(64, 48, 100, *wpt.scenes.scene_camera(100))
    try:
        for name, v in list(cases()) + list(walk_cases()):
            assert same(seq(v), device(wpt, v)), (name, seq(v), device(wpt, v))
        rng = np.random.default_rng(23)
        for t in range(40):
            n = int(rng.integers(0, 200000))
            v = (rng.exponential(1.0, n) * 10.0 ** rng.integers(-20, 5)).astype(np.float32)
            assert same(seq(v), device(wpt, v)), t
    finally:
        itf.shutdown()

"""Committed golden vectors (tests/golden/golden.npz, made by
tests/golden/make_golden.py from the oracle): the oracle must still reproduce
them (CPU), and the HIP path must match them bit for bit (GPU) — the GPU
check needs no oracle at run time."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)  # allow_pickle=False (default)


def _images(g):
    i = 0
    while f"img{i}_cfg" in g:
        yield i, [int(v) for v in g[f"img{i}_cfg"]], g[f"img{i}_acc"]
        i += 1


def _cloud(wpt, g):
    n, seed = (int(v) for v in g["cloud_params"])
    return wpt.scenes.triangle_cloud(n, seed=seed)


def test_oracle_reproduces_golden(wpt, oracle, golden):
    cloud = _cloud(wpt, golden)
    seed = int(golden["seed"][0])
    for i, (sid, w, h, spp, depth, lt, rt), acc in _images(golden):
        sc = oracle.OracleScene(sid, cloud if sid == 2 else None)
        got, _ = sc.render(w, h, wpt.scenes.scene_camera(sid), lt, rt, depth, seed, 0, spp, threads=4)
        assert np.array_equal(got.view(np.uint32), acc.view(np.uint32)), f"image {i}"
    for sid in (2, 100, 101):
        sc = oracle.OracleScene(sid, cloud if sid == 2 else None)
        t, ids, _ = sc.trace_rays(golden[f"hits{sid}_rays"])
        assert np.array_equal(ids, golden[f"hits{sid}_id"])
        assert np.array_equal(t.view(np.uint32), golden[f"hits{sid}_t"].view(np.uint32))


@pytest.mark.gpu
def test_gpu_matches_golden_images(wpt, golden):
    itf = wpt.interface
    cloud = _cloud(wpt, golden)
    seed = int(golden["seed"][0])
    try:
        for i, (sid, w, h, spp, depth, lt, rt), acc in _images(golden):
            itf.init(w, h, sid, *wpt.scenes.scene_camera(sid))
            if sid == 2:
                itf.store_mesh(1, cloud)
            itf.update_settings(lt, rt, 0, 0, 0)
            itf.set_render_options(depth, seed, 0)
            itf.compute(w * h * spp)
            got, cnt = itf.read_radiance(w, h)
            assert np.all(cnt == spp)
            assert np.array_equal(got.view(np.uint32), acc.view(np.uint32)), f"image {i}"
            itf.shutdown()
    finally:
        try:
            itf.shutdown()
        except itf.WptError:
            pass


@pytest.mark.gpu
def test_gpu_matches_golden_hits(wpt, golden):
    itf = wpt.interface
    cloud = _cloud(wpt, golden)
    try:
        for sid in (2, 100, 101):
            itf.init(16, 16, sid, *wpt.scenes.scene_camera(sid))
            if sid == 2:
                itf.store_mesh(1, cloud)
            t, ids = itf.trace_rays(golden[f"hits{sid}_rays"])
            assert np.array_equal(ids, golden[f"hits{sid}_id"])
            assert np.array_equal(t.view(np.uint32), golden[f"hits{sid}_t"].view(np.uint32))
            itf.shutdown()
    finally:
        try:
            itf.shutdown()
        except itf.WptError:
            pass

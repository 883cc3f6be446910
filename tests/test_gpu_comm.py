"""The product's own RCCL path (wpt_set_comm / wpt_gather_frame, SURVEY.md
§8e): what a Rust host calls to render across the GPUs of a node with no
Python in between. The 1-GPU development box can run world size 1 (the
communicator's set-up, the gather's pack / unpack and the adaptive exchange
hook) and, when RCCL accepts two ranks on one device, world size 2 over the
real collective."""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, DEPTH, TILE = 40, 24, 3, 4, 8


def _setup(itf, scenes, adaptive=False):
    itf.set_device(0)
    itf.init(W, H, 2, *scenes.scene_camera(2))
    itf.store_mesh(1, scenes.triangle_cloud(2000, seed=0xC0))
    itf.update_settings(1, 2 if adaptive else 1, int(adaptive), int(adaptive), 0)
    itf.set_render_options(DEPTH, 0xBABABEBE, 0)


@pytest.mark.parametrize("adaptive", [False, True])
def test_comm_world_one(wpt, adaptive):
    itf = wpt.interface
    _setup(itf, wpt.scenes, adaptive)
    try:
        itf.compute(W * H * SPP)
        ref_acc, ref_cnt = itf.read_radiance(W, H)
    finally:
        itf.shutdown()
    _setup(itf, wpt.scenes, adaptive)
    try:
        itf.set_comm(0, 1, TILE, itf.comm_unique_id())
        itf.compute(W * H * SPP)
        itf.gather_frame(0)
        acc, cnt = itf.read_radiance(W, H)
        with pytest.raises(itf.WptError):
            itf.gather_frame(1)  # no such rank
        itf.comm_destroy()
    finally:
        itf.shutdown()
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))


def test_comm_survives_viewport_growth(wpt):
    """The communicator's buffers follow the partition when the viewport
    grows after wpt_set_comm (update_viewport keeps the partition)."""
    itf = wpt.interface
    W2, H2 = 2 * W + 6, 2 * H + 4
    _setup(itf, wpt.scenes)
    try:
        itf.update_viewport(W2, H2)
        itf.compute(W2 * H2 * SPP)
        ref_acc, ref_cnt = itf.read_radiance(W2, H2)
    finally:
        itf.shutdown()
    _setup(itf, wpt.scenes)
    try:
        itf.set_comm(0, 1, TILE, itf.comm_unique_id())
        itf.update_viewport(W2, H2)
        itf.compute(W2 * H2 * SPP)
        itf.gather_frame(0)
        acc, cnt = itf.read_radiance(W2, H2)
        itf.comm_destroy()
    finally:
        itf.shutdown()
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))


def _rank(rank, world, uid_q, out_q, adaptive):
    sys.path.insert(0, ROOT)
    try:
        import wpt_loader
        pkg = wpt_loader.load()
        itf = pkg.interface
        _setup(itf, pkg.scenes, adaptive)
        if rank == 0:
            uid = itf.comm_unique_id()
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        itf.set_comm(rank, world, TILE, uid)
        itf.compute(W * H * SPP)
        itf.gather_frame(0)
        acc, cnt = itf.read_radiance(W, H)
        out_q.put((rank, "ok", acc if rank == 0 else None, cnt if rank == 0 else None))
        itf.comm_destroy()
        itf.shutdown()
    except Exception as e:  # reported to the test
        out_q.put((rank, f"{type(e).__name__}: {e}", None, None))


@pytest.mark.parametrize("adaptive", [False, True])
def test_comm_two_ranks_one_gpu(wpt, adaptive):
    itf = wpt.interface
    _setup(itf, wpt.scenes, adaptive)
    try:
        itf.compute(W * H * SPP)
        ref_acc, ref_cnt = itf.read_radiance(W, H)
    finally:
        itf.shutdown()
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, uid_q, out_q, adaptive)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, status, acc, cnt = out_q.get(timeout=150)
            res[r] = (status, acc, cnt)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    if any("ncclCommInitRank" in s for s, _, _ in res.values()):
        pytest.skip(f"RCCL refuses two ranks on one GPU here: {res}")
    assert all(s == "ok" for s, _, _ in res.values()), res
    _, acc, cnt = res[0]
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))

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
        # random halves: this rank's share of the rounds; adaptive: the global n
        itf.compute(W * H * SPP if adaptive else len(itf.partition_pixels()) * SPP)
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


def _transport_rank(rank, world, port, adaptive, chunks, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import wpt_loader
        pkg = wpt_loader.load()
        from wasm_pathtracer_amd import multigpu
        itf = pkg.interface
        _setup(itf, pkg.scenes, adaptive)
        itf.set_partition(rank, world, TILE)
        xf = multigpu.Transport(world, rank, device="cuda")
        npart = len(itf.partition_pixels())
        for n in chunks:
            # random halves: compute(n) traces n paths over this rank's own
            # pixels (n = its share of whole rounds); adaptive halves: n
            # positions of the GLOBAL round sequence, the same n on every rank
            itf.compute(n if adaptive else n * npart // (W * H))
        itf.gather_frame(0)  # pack -> the transport's gather -> root unpacks
        acc, cnt = itf.read_radiance(W, H)
        calls = dict(xf.calls)
        xf.close()
        with pytest.raises(itf.WptError):
            itf.gather_frame(0)  # no transport, no communicator
        q.put((rank, "ok", acc if rank == 0 else None, cnt if rank == 0 else None, calls))
        itf.shutdown()
    except Exception as e:  # reported to the test
        q.put((rank, f"{type(e).__name__}: {e}", None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,adaptive", [(2, False), (3, False), (2, True), (3, True)])
def test_transport_gather_multirank(wpt, world, adaptive):
    """wpt_gather_frame over a caller transport (wpt_set_transport) at world
    size 2 and 3: one process per rank on this GPU (gloo, staged through host
    memory), each tracing its interleaved-tile partition. The library packs,
    the transport moves the rank-major buffers, rank 0 unpacks: rank 0's frame
    must be the single-rank frame bit for bit. With adaptive halves the round
    boundaries' frame exchange goes through the same transport (ALLGATHER)."""
    import socket

    import torch.multiprocessing as tmp

    chunks = (W * H * SPP,) if not adaptive else (1500, 2200, 700)
    itf = wpt.interface
    _setup(itf, wpt.scenes, adaptive)
    try:
        for n in chunks:
            itf.compute(n)
        ref_acc, ref_cnt = itf.read_radiance(W, H)
    finally:
        itf.shutdown()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = tmp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = tmp.start_processes(_transport_rank, args=(world, port, adaptive, chunks, q), nprocs=world, join=False,
                             start_method="spawn")
    import time
    deadline = time.time() + 200
    while not pc.join(timeout=5):
        if time.time() > deadline:
            for p in pc.processes:
                p.kill()
            raise TimeoutError("transport ranks did not finish")
    res = {}
    for _ in range(world):
        r, status, acc, cnt, calls = q.get()
        res[r] = (status, acc, cnt, calls)
    assert all(v[0] == "ok" for v in res.values()), res
    _, acc, cnt, calls = res[0]
    assert calls[0] == 1  # one gather
    assert (calls[1] > 0) == adaptive  # adaptive rounds exchanged the frame through it
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))

"""Adaptive sampling over several ranks (SURVEY.md §8e, C5 on N GPUs).

Two ranks share the box's one GPU (one process each, gloo process group; the
round-boundary frame exchange is staged through host memory, the same
callback bench.py runs over RCCL). Each rank renders its interleaved-tile
partition with adaptive halves (PNEE on one half) through compute() calls that
cut rounds at arbitrary points; the union of the partitions must equal the
single-rank frame bit for bit — sample counts, radiance and the sampling view
(which every rank plans for the whole frame).
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, DEPTH, TILE = 48, 32, 4, 8
CHUNKS = (1500, 4000, 6100, 9000)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(itf, scenes, scene_id, types, adaptive, batch):
    cam = scenes.scene_camera(scene_id)
    itf.set_device(0)
    itf.init(W, H, scene_id, *cam)
    if scene_id == 2:
        itf.store_mesh(1, scenes.triangle_cloud(3000, seed=0x5EED))
    itf.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
    itf.set_render_options(DEPTH, 0xBABABEBE, batch)


def _worker(rank, world, port, scene_id, types, adaptive, batch, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import wpt_loader
        pkg = wpt_loader.load()
        from wasm_pathtracer_amd import multigpu
        itf = pkg.interface
        _setup(itf, pkg.scenes, scene_id, types, adaptive, batch)
        itf.set_partition(rank, world, TILE)
        ex = multigpu.RoundExchange(world, device="cuda")
        for n in CHUNKS:
            itf.compute(n)
        px = itf.partition_pixels()
        acc, cnt = itf.read_radiance(W, H)
        samp = itf.results(1, W, H)
        q.put((rank, px, acc.reshape(-1, 3)[px], cnt.reshape(-1)[px], samp, ex.calls, itf.stats()["paths"]))
        ex.close()
        itf.shutdown()
    finally:
        dist.destroy_process_group()


def _run_ranks(world, args, timeout_s=240):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_worker, args=(world, _free_port(), *args, q), nprocs=world, join=False,
                            start_method="spawn")
    deadline = time.time() + timeout_s
    while not pc.join(timeout=5):
        if time.time() > deadline:
            for p in pc.processes:
                p.kill()
            raise TimeoutError("multi-rank workers did not finish")
    return sorted((q.get() for _ in range(world)), key=lambda r: r[0])


@pytest.mark.parametrize("scene_id,types,adaptive,batch,world", [
    (2, (2, 1), (1, 1), 0, 2),      # C5-like: PNEE + NEE halves, both adaptive
    (2, (1, 1), (0, 1), 900, 2),    # one adaptive half, small batches
    (101, (1, 1), (1, 0), 0, 3),    # BVH-less scene, three ranks
])
def test_adaptive_multirank_bitwise(wpt, scene_id, types, adaptive, batch, world):
    itf = wpt.interface
    _setup(itf, wpt.scenes, scene_id, types, adaptive, batch)
    try:
        for n in CHUNKS:
            itf.compute(n)
        ref_acc, ref_cnt = itf.read_radiance(W, H)
        ref_samp = itf.results(1, W, H)
    finally:
        itf.shutdown()
    res = _run_ranks(world, (scene_id, types, adaptive, batch))
    acc = np.zeros((W * H, 3), np.float32)
    cnt = np.zeros(W * H, np.uint32)
    seen = np.zeros(W * H, np.int32)
    paths = 0
    for rank, px, a, c, samp, calls, npaths in res:
        acc[px] = a
        cnt[px] = c
        seen[px] += 1
        paths += npaths
        assert calls > 0  # rounds past the first exchanged the frame
        assert np.array_equal(samp, ref_samp), f"rank {rank}: sampling view differs"
    assert np.all(seen == 1)
    assert paths == sum(CHUNKS)
    assert ref_cnt.max() > 4
    assert np.array_equal(cnt, ref_cnt.reshape(-1))
    assert np.array_equal(acc.view(np.uint32), ref_acc.reshape(-1, 3).view(np.uint32))

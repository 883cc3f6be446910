"""Multi-process (gloo, CPU) test of the multi-GPU path's data movement
(SURVEY.md §8e): interleaved-tile partitions from the C ABI, one gather of the
packed float4 partitions to rank 0 (multigpu.FrameGather — the same code
bench.py runs over RCCL), scatter into the frame. Each rank's partition
radiance comes from the oracle's full-frame render, so rank 0's assembled
frame must equal that render bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, tile, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pyoracle
        import wpt_loader
        pkg = wpt_loader.load()
        from wasm_pathtracer_amd import multigpu
        cloud = pkg.scenes.triangle_cloud(500, seed=7)
        acc, _ = pyoracle.OracleScene(2, cloud).render(W, H, pkg.scenes.scene_camera(2), 1, 1, 4, 0xBABABEBE, 0, 2,
                                                       threads=1)
        g = multigpu.FrameGather(W, H, rank, world, tile)
        px = g.parts[rank].numpy()
        cnt = np.full(len(px), 2, np.uint32)  # sample counts travel as u32 bits (wpt_copy_partition)
        local = np.concatenate([acc.reshape(-1, 3)[px], cnt.view(np.float32)[:, None]], axis=1)
        g.local_view().copy_(torch.from_numpy(local))
        frame = g.gather()
        if rank == 0:
            f = frame.numpy()
            q.put((bool(np.array_equal(f[..., :3].view(np.uint32), acc.view(np.uint32))),
                   bool(np.all(np.ascontiguousarray(f[..., 3]).view(np.uint32) == 2))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,tile", [(2, 40, 24, 8), (3, 37, 21, 16)])
def test_gloo_frame_gather(world, W, H, tile):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), W, H, tile, q), nprocs=world, join=True,
                       start_method="spawn")
    same, counts = q.get()
    assert same and counts


def test_partitions_cover_frame_once(wpt):
    for world in (1, 2, 4, 8):
        W, H = 1920, 1080
        parts = [wpt.interface.tile_partition(W, H, r, world, 16) for r in range(world)]
        allp = np.sort(np.concatenate(parts))
        assert np.array_equal(allp, np.arange(W * H, dtype=np.uint32))
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 16 * 16 * 2  # balanced to within ~one tile per rank


def _xworker(rank, world, port, W, H, tile, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pyoracle
        import wpt_loader
        pkg = wpt_loader.load()
        from wasm_pathtracer_amd import multigpu
        cloud = pkg.scenes.triangle_cloud(400, seed=3)
        acc, _ = pyoracle.OracleScene(2, cloud).render(W, H, pkg.scenes.scene_camera(2), 1, 1, 3, 0xBABABEBE, 0, 1,
                                                       threads=1)
        parts = [pkg.interface.tile_partition(W, H, r, world, tile).astype(np.int64) for r in range(world)]
        slot = max(len(p) for p in parts)
        px = parts[rank]
        cnt = (np.arange(W * H, dtype=np.uint32) * 7 + 1 + (1 << 25))  # exact past 2^24: u32 bits
        local = torch.zeros((slot, 4), dtype=torch.float32)
        lv = np.concatenate([acc.reshape(-1, 3)[px], cnt[px].view(np.float32)[:, None]], axis=1)
        local[: len(px)] = torch.from_numpy(lv)
        gathered = torch.zeros((world * slot, 4), dtype=torch.float32)
        multigpu.all_gather_slots(local, gathered, world, staged=True)
        fa = np.zeros_like(acc)
        fc = np.zeros(W * H, np.uint32)
        multigpu.scatter_slots(gathered.numpy(), parts, slot, fa, fc)
        q.put((rank, bool(np.array_equal(fa.view(np.uint32), acc.view(np.uint32))), bool(np.array_equal(fc, cnt))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,tile", [(2, 40, 24, 8), (3, 37, 21, 16)])
def test_gloo_round_exchange(world, W, H, tile):
    """The adaptive-round frame exchange (multigpu.all_gather_slots, the
    callback behind wpt_set_exchange): every rank ends with the whole frame."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_xworker, args=(world, _free_port(), W, H, tile, q), nprocs=world, join=True,
                       start_method="spawn")
    res = sorted(q.get() for _ in range(world))
    assert [r[0] for r in res] == list(range(world))
    assert all(r[1] and r[2] for r in res), res


@pytest.mark.parametrize("nranks,root", [(1, 0), (2, 0), (3, 1), (8, 0), (8, 5)])
def test_gather_plan_offsets(nranks, root):
    """wpt_gather_frame's point-to-point plan (wpt_comm.cpp gather_plan, the
    grouped ncclSend / ncclRecv): the root receives every other rank's slot at
    offset rank * slot of its rank-major buffer, every other rank sends its
    one slot to the root, and the sends and receives pair up one to one."""
    sys.path.insert(0, ROOT)
    import wpt_loader
    itf = wpt_loader.load().interface
    slot = 1037
    recvs, sends = {}, {}
    for r in range(nranks):
        ops = itf.gather_plan(r, nranks, root, slot)
        if r == root:
            assert all(rc for _, _, _, rc in ops)
            assert len(ops) == nranks - 1
            for peer, off, cnt, _ in ops:
                assert peer != root and cnt == slot and off == peer * slot
                recvs[peer] = off
        else:
            assert ops == [(root, 0, slot, False)]
            sends[r] = root
    assert sorted(recvs) == sorted(sends) == [r for r in range(nranks) if r != root]
    # the received slots tile the root's buffer without overlap (its own slot stays free)
    spans = sorted((off, off + slot) for off in recvs.values())
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    with pytest.raises(itf.WptError):
        itf.gather_plan(0, nranks, nranks, slot)  # root out of range

"""Multi-GPU frame assembly: one process per GPU, each
rendering its interleaved-tile partition (wpt_set_partition), then ONE gather
of the packed partitions to rank 0 over torch.distributed (RCCL on the GPU,
gloo in the CPU tests) and a scatter into the full frame.

Packed partition layout (wpt_copy_partition): float4 per partition pixel =
(acc.x, acc.y, acc.z, sample count as u32 bits), in partition order — the
same layout as the adaptive-round exchange; read the count with
``frame[..., 3].view(torch.int32)``. Ranks send buffers
padded to the largest partition; rank 0 knows every rank's pixel list from
the host-only wpt_tile_partition, so no indices travel.
"""
import torch
import torch.distributed as dist

from . import interface


class FrameGather:
    """Pre-sized buffers and index maps for gathering partitions on `dst`."""

    def __init__(self, width, height, rank, world, tile=16, device="cpu", dst=0):
        self.w, self.h, self.rank, self.world, self.dst = width, height, rank, world, dst
        self.parts = [torch.from_numpy(interface.tile_partition(width, height, r, world, tile).astype("int64"))
                      for r in range(world)]
        self.maxpart = max(len(p) for p in self.parts)
        self.npart = len(self.parts[rank])
        self.device = torch.device(device)
        self.send = torch.zeros((self.maxpart, 4), dtype=torch.float32, device=self.device)
        if rank == dst:
            self.recv = [torch.empty_like(self.send) for _ in range(world)]
            self.index = [p.to(self.device) for p in self.parts]
            self.frame = torch.zeros((height * width, 4), dtype=torch.float32, device=self.device)
        else:
            self.recv = None

    def local_view(self):
        """The first npart rows of the send buffer (wpt_copy_partition target)."""
        return self.send[: self.npart]

    def gather(self):
        """Collective: every rank calls it; rank dst returns the (H, W, 4) frame.
        With a gloo group and device buffers (a multi-rank rehearsal on one
        GPU) the gather is staged through host memory."""
        if self.device.type == "cuda" and dist.get_backend() != "nccl":
            recv = [torch.empty_like(self.send, device="cpu") for _ in range(self.world)] if self.recv else None
            dist.gather(self.send.cpu(), recv, dst=self.dst)
            if recv is not None:
                for r in range(self.world):
                    self.recv[r].copy_(recv[r])
        else:
            dist.gather(self.send, self.recv, dst=self.dst)
        if self.rank != self.dst:
            return None
        for r in range(self.world):
            self.frame.index_copy_(0, self.index[r], self.recv[r][: len(self.parts[r])])
        return self.frame.view(self.h, self.w, 4)


def all_gather_slots(local, gathered, world, staged=False):
    """All-gather every rank's ``local`` (slot, 4) buffer into ``gathered``
    (world * slot, 4), rank-major; ``staged`` goes through host memory (gloo).
    Returns once the data is in place (device synchronised)."""
    if staged:
        loc = local.cpu()
        out = [torch.empty_like(loc) for _ in range(world)]
        dist.all_gather(out, loc)
        gathered.copy_(torch.cat(out).to(gathered.device))
    else:
        dist.all_gather_into_tensor(gathered, local)
    if gathered.device.type == "cuda":
        torch.cuda.synchronize(gathered.device)


def scatter_slots(gathered, parts, slot, frame_acc, frame_cnt):
    """Host restatement of k_unpack_exchange: entry j of rank r's slot is
    pixel parts[r][j] (acc.xyz, count as u32 bits). Test helper."""
    import numpy as np

    g = np.asarray(gathered).reshape(len(parts), slot, 4)
    for r, px in enumerate(parts):
        frame_acc.reshape(-1, 3)[px] = g[r, : len(px), :3]
        frame_cnt.reshape(-1)[px] = g[r, : len(px), 3].view(np.uint32)


class RoundExchange:
    """Frame exchange of adaptive sample rounds over several ranks
    (wpt_set_exchange): at each round boundary libwpt packs this
    rank's partition into ``local`` and calls back; the callback all-gathers
    every rank's buffer into ``gathered`` (rank-major), after which every rank
    holds the whole frame and plans the same global round.

    The buffers live on the rank's GPU. With a ``nccl`` (RCCL) group the
    all-gather runs device to device; with ``gloo`` (the single-GPU box's
    multi-process tests) it is staged through host memory.
    """

    def __init__(self, world, device="cuda"):
        import ctypes

        from ._lib import lib

        L = lib()
        slot = L.wpt_exchange_slot()
        if slot < 0:
            raise interface.WptError(slot, L.wpt_last_error().decode())
        self.slot, self.world = int(slot), world
        self.device = torch.device(device)
        self.local = torch.zeros((self.slot, 4), dtype=torch.float32, device=self.device)
        self.gathered = torch.zeros((world * self.slot, 4), dtype=torch.float32, device=self.device)
        self.calls = 0
        self.host = dist.get_backend() != "nccl"

        def _fn(_user):
            try:
                self._exchange()
                return 0
            except Exception as e:  # reported through wpt_last_error as "frame exchange failed"
                self.error = e
                return 1

        self.error = None
        self._cb = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)(_fn)  # kept alive with self
        rc = L.wpt_set_exchange(ctypes.cast(self._cb, ctypes.c_void_p), None, self.local.data_ptr(), self.gathered.data_ptr(), self.slot)
        if rc < 0:
            raise interface.WptError(rc, L.wpt_last_error().decode())

    def _exchange(self):
        self.calls += 1
        all_gather_slots(self.local, self.gathered, self.world, staged=self.host)

    def close(self):
        from ._lib import lib

        lib().wpt_set_exchange(None, None, None, None, 0)


XFER_GATHER, XFER_ALLGATHER = 0, 1  # include/wpt.h


class Transport:
    """A caller transport for libwpt's multi-rank data movement
    (wpt_set_transport): the library packs this rank's partition into
    ``send`` and calls back; the callback moves the rank-major buffers with
    torch.distributed (device to device over RCCL, staged through host
    memory over gloo), and the library unpacks ``recv`` into the frame.
    op GATHER (wpt_gather_frame): every rank's ``send`` into root's ``recv``;
    op ALLGATHER (adaptive round boundaries): into every rank's. Call after
    wpt_set_partition; the slot is the largest partition (wpt_exchange_slot).
    """

    def __init__(self, world, rank, device="cuda"):
        import ctypes

        from ._lib import lib

        L = lib()
        slot = L.wpt_exchange_slot()
        if slot < 0:
            raise interface.WptError(slot, L.wpt_last_error().decode())
        self.slot, self.world, self.rank = max(int(slot), 1), world, rank
        self.device = torch.device(device)
        self.send = torch.zeros((self.slot, 4), dtype=torch.float32, device=self.device)
        self.recv = torch.zeros((world * self.slot, 4), dtype=torch.float32, device=self.device)
        self.host = dist.get_backend() != "nccl"
        self.calls = {XFER_GATHER: 0, XFER_ALLGATHER: 0}
        self.error = None

        def _fn(_user, op, root):
            try:
                self._move(int(op), int(root))
                return 0
            except Exception as e:  # surfaces as the call's WptError
                self.error = e
                return 1

        self._cb = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32)(_fn)
        rc = L.wpt_set_transport(ctypes.cast(self._cb, ctypes.c_void_p), None, self.send.data_ptr(),
                                 self.recv.data_ptr(), self.slot)
        if rc < 0:
            raise interface.WptError(rc, L.wpt_last_error().decode())

    def _move(self, op, root):
        self.calls[op] += 1
        if op == XFER_ALLGATHER:
            all_gather_slots(self.send, self.recv, self.world, staged=self.host)
            return
        if op != XFER_GATHER:
            raise ValueError(f"unknown transport op {op}")
        if self.host:
            loc = self.send.cpu()
            out = [torch.empty_like(loc) for _ in range(self.world)] if self.rank == root else None
            dist.gather(loc, out, dst=root)
            if out is not None:
                self.recv.copy_(torch.cat(out).to(self.device))
        else:
            out = list(self.recv.view(self.world, self.slot, 4).unbind(0)) if self.rank == root else None
            dist.gather(self.send, out, dst=root)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def close(self):
        from ._lib import lib

        lib().wpt_set_transport(None, None, None, None, 0)

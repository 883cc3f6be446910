"""Multi-GPU frame assembly: one process per GPU, each
rendering its interleaved-tile partition (wpt_set_partition), then ONE gather
of the packed partitions to rank 0 over torch.distributed (RCCL on the GPU,
gloo in the CPU tests) and a scatter into the full frame.

Packed partition layout (wpt_copy_partition): float4 per partition pixel =
(acc.x, acc.y, acc.z, sample count), in partition order. Ranks send buffers
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
        """Collective: every rank calls it; rank dst returns the (H, W, 4) frame."""
        dist.gather(self.send, self.recv, dst=self.dst)
        if self.rank != self.dst:
            return None
        for r in range(self.world):
            self.frame.index_copy_(0, self.index[r], self.recv[r][: len(self.parts[r])])
        return self.frame.view(self.h, self.w, 4)

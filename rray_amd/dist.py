"""Multi-GPU tiling: one process per GPU, row-interleaved tiles, one gather to rank 0.

Pixels are independent (camera.rs:110-118 renders them in any order), so rank r renders the output
rows {y : (y // block) % N == r} (interleaved blocks balance sky/floor cost) and one collective
(torch.distributed.gather; backend "nccl" is RCCL over xGMI on ROCm, "gloo" on CPU tests) brings
the tiles to rank 0, which scatters the rows back into frame order.  The gather buffer layout and the
un-interleave are the library's (partition.hpp, rr_unshuffle_host): the same runs as the C ABI's own
multi-GPU path places (multi.cpp), so CPU rehearsals of this module exercise that arithmetic.

FramePipeline double-buffers the tiles so that rendering frame k+1 overlaps the gather of frame k
(the gather runs on the process group's own stream; the renderer waits only for the gather that
last read the buffer it is about to overwrite).
"""
import numpy as np
import torch
import torch.distributed as dist

from .render import part_rows, unshuffle


def tile_rows(height, rank, world, block=8):
    return part_rows(height, rank, world, block)


def max_tile_rows(height, world, block=8):
    """Padded rows per tile in the gather buffer (part 0 holds the most rows; partition.hpp)."""
    return len(part_rows(height, 0, world, block))


def gather_sources(height, world, block=8):
    """For every output row y, its row in the gathered buffer (world tiles of max_tile_rows rows back
    to back, torch.distributed.gather's layout), computed by the library's own run placement
    (rr_unshuffle_host, the runs of multi.cpp's transfer) applied to a buffer whose rows hold their indices."""
    rows = max_tile_rows(height, world, block)
    idx = np.repeat(np.arange(world * rows, dtype=np.float64), 3).reshape(world * rows, 1, 3)
    return unshuffle(idx, height, world, block)[:, 0, 0].astype(np.int64)


def gather_frame(tile, height, block=8, dst=0, group=None, out=None):
    """tile: (max_tile_rows, W, C) with this rank's rows first (padding after).  One gather into a
    contiguous (world * max_tile_rows, W, C) buffer on `dst`, then the library's run placement
    (rr_unshuffle_host: the runs multi.cpp's receives place on the device).  Returns the (height, W, C) frame on `dst` (written
    into `out` when given), None on the other ranks."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    big = torch.empty((world,) + tuple(tile.shape), dtype=tile.dtype, device=tile.device) if rank == dst else None
    dist.gather(tile, gather_list=list(big.unbind(0)) if big is not None else None, dst=dst, group=group)
    if rank != dst:
        return None
    flat = big.view(world * tile.shape[0], *tile.shape[1:])
    if tile.device.type == "cpu" and tile.dtype == torch.float64 and tile.shape[-1] == 3:
        frame = torch.from_numpy(unshuffle(flat.numpy(), height, world, block))  # rr_unshuffle_host
    else:
        src = torch.as_tensor(gather_sources(height, world, block), device=tile.device)
        frame = torch.index_select(flat, 0, src)
    if out is not None:
        out.copy_(frame)
        return out
    return frame


class FramePipeline:
    """Double-buffered tiles + one async gather per frame to `dst`, reassembled with a single
    index_select.  Usage per frame: i, tile, prev = pipe.acquire(); (make the render stream wait on
    `prev` if not None, render into `tile`, make the current stream wait for the render); then
    pipe.submit(i).  pipe.frame holds the latest assembled frame on `dst` once its gather is done."""

    def __init__(self, height, width, channels, dtype, device, block=8, dst=0, group=None, depth=2):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst, self.group, self.depth = dst, group, depth
        self.rows = max_tile_rows(height, self.world, block)
        shape = (self.rows, width, channels)
        self.tiles = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(depth)]
        self.pending = [None] * depth
        self.k = 0
        self.frame = None
        if self.rank == dst:
            self.big = torch.empty((self.world,) + shape, dtype=dtype, device=device)
            self.gl = list(self.big.unbind(0))
            self.src = torch.as_tensor(gather_sources(height, self.world, block), dtype=torch.long, device=device)
            self.frame = torch.empty((height, width, channels), dtype=dtype, device=device)

    def acquire(self):
        i = self.k % self.depth
        return i, self.tiles[i], self.pending[i]

    def submit(self, i):
        root = self.rank == self.dst
        work = dist.gather(self.tiles[i], gather_list=self.gl if root else None, dst=self.dst, group=self.group,
                           async_op=True)
        self.pending[i] = work
        if root:  # the current stream waits for the gather, then un-interleaves into the frame
            work.wait()
            torch.index_select(self.big.view(self.world * self.rows, *self.big.shape[2:]), 0, self.src,
                               out=self.frame)
        self.k += 1

    def drain(self):
        for w in self.pending:
            if w is not None:
                w.wait()

"""Multi-GPU tiling: one process per GPU, row-interleaved tiles, one gather to rank 0.

Pixels are independent (camera.rs:110-118 renders them in any order), so rank r renders the output
rows {y : (y // block) % N == r} (interleaved blocks balance sky/floor cost) and one collective
(torch.distributed.gather; backend "nccl" is RCCL over xGMI on ROCm, "gloo" on CPU tests) brings
the tiles to rank 0, which scatters the rows back into frame order.

FramePipeline double-buffers the tiles so that rendering frame k+1 overlaps the gather of frame k
(the gather runs on the process group's own stream; the renderer waits only for the gather that
last read the buffer it is about to overwrite).
"""
import torch
import torch.distributed as dist

from .render import part_rows


def tile_rows(height, rank, world, block=8):
    return part_rows(height, rank, world, block)


def max_tile_rows(height, world, block=8):
    return max(len(part_rows(height, p, world, block)) for p in range(world))


def gather_frame(tile, height, block=8, dst=0, group=None, out=None):
    """tile: (max_tile_rows, W, C) with this rank's rows first.  Returns the (height, W, C) frame on
    `dst` (written into `out` when given), None on the other ranks."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    gl = [torch.empty_like(tile) for _ in range(world)] if rank == dst else None
    dist.gather(tile, gather_list=gl, dst=dst, group=group)
    if rank != dst:
        return None
    frame = out if out is not None else torch.empty((height,) + tuple(tile.shape[1:]), dtype=tile.dtype,
                                                      device=tile.device)
    for p in range(world):
        rows = torch.as_tensor(part_rows(height, p, world, block), device=tile.device)
        frame.index_copy_(0, rows, gl[p][: len(rows)])
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
            src = [0] * height
            for p in range(self.world):
                for j, y in enumerate(part_rows(height, p, self.world, block)):
                    src[y] = p * self.rows + j
            self.src = torch.as_tensor(src, dtype=torch.long, device=device)
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

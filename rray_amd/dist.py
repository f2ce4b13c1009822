"""Multi-GPU tiling through torch.distributed: one process per GPU, row-interleaved tiles, one point-to-point
transfer per part to rank 0.

Pixels are independent (camera.rs:110-118 renders them in any order), so rank r renders the output
rows {y : (y // block) % N == r} (interleaved blocks balance sky/floor cost).  The transfer mirrors the
library's own (multi.cpp): every rank sends its whole, unpadded tile to rank 0 (backend "nccl" is RCCL over
xGMI on ROCm, "gloo" on CPU tests), and rank 0 receives part p's tile into a staging buffer of `height`
rows at row stage_row_offset(p) — its own tile by a local copy (torch.distributed refuses a send to oneself;
the library sends to itself) — then moves each tile's runs into their frame rows.  The staging layout and
the un-interleave are the library's (partition.hpp: rr_stage_row_offset, rr_unshuffle_host), so CPU
rehearsals of this module exercise the arithmetic the device placement kernels run.

FramePipeline double-buffers the tiles so that rendering frame k+1 overlaps the transfer of frame k
(the renderer waits only for the send that last read the buffer it is about to overwrite).
"""
import numpy as np
import torch
import torch.distributed as dist

from .render import part_rows, stage_row_offset, unshuffle


def tile_rows(height, rank, world, block=8):
    return part_rows(height, rank, world, block)


def stage_sources(height, world, block=8):
    """For every output row y, its row in the staging buffer (the parts' tiles back to back, unpadded), computed
    by the library's own run placement (rr_unshuffle_host) applied to a buffer whose rows hold their indices."""
    idx = np.repeat(np.arange(height, dtype=np.float64), 3).reshape(height, 1, 3)
    return unshuffle(idx, height, world, block)[:, 0, 0].astype(np.int64)


def _post_transfer(tile, stage, height, block, dst, group):
    """One send per part to `dst` (its own part: a local copy); on `dst`, one receive per other part into its
    stage rows.  Returns the pending operations."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ops = []
    if rank != dst:
        if tile.shape[0] > 0:
            ops.append(dist.isend(tile, dst=dst, group=group))
        return ops
    for p in range(world):
        off = stage_row_offset(height, p, world, block)
        n = stage_row_offset(height, p + 1, world, block) - off
        if n == 0:
            continue
        if p == rank:
            stage[off:off + n].copy_(tile[:n])
        else:
            ops.append(dist.irecv(stage[off:off + n], src=p, group=group))
    return ops


def _assemble(stage, height, world, block, src=None, out=None):
    if stage.device.type == "cpu" and stage.dtype == torch.float64 and stage.shape[-1] == 3:
        frame = torch.from_numpy(unshuffle(stage.numpy(), height, world, block))  # rr_unshuffle_host
    else:
        if src is None:
            src = torch.as_tensor(stage_sources(height, world, block), device=stage.device)
        frame = torch.index_select(stage, 0, src)
    if out is not None:
        out.copy_(frame)
        return out
    return frame


def gather_frame(tile, height, block=8, dst=0, group=None, out=None):
    """tile: (tile_rows(height, rank, world, block), W, C), this rank's rows in increasing y.  Every rank sends
    its tile to `dst`, which receives each into its staging rows and places the runs (rr_unshuffle_host).
    Returns the (height, W, C) frame on `dst` (written into `out` when given), None on the other ranks."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    stage = torch.empty((height,) + tuple(tile.shape[1:]), dtype=tile.dtype, device=tile.device) if rank == dst \
        else None
    for op in _post_transfer(tile, stage, height, block, dst, group):
        op.wait()
    if rank != dst:
        return None
    return _assemble(stage, height, world, block, out=out)


class FramePipeline:
    """Double-buffered tiles + one asynchronous per-part transfer per frame to `dst`, reassembled with a single
    index_select.  Usage per frame: i, tile, prev = pipe.acquire(); (make the render stream wait on
    `prev` if not None, render into `tile`, make the current stream wait for the render); then
    pipe.submit(i).  pipe.frame holds the latest assembled frame on `dst` once its transfer is done."""

    def __init__(self, height, width, channels, dtype, device, block=8, dst=0, group=None, depth=2):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.height, self.block = height, block
        self.dst, self.group, self.depth = dst, group, depth
        self.rows = len(tile_rows(height, self.rank, self.world, block))
        shape = (self.rows, width, channels)
        self.tiles = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(depth)]
        self.pending = [None] * depth
        self.k = 0
        self.frame = None
        self.stage = None
        if self.rank == dst:
            self.stage = torch.empty((height, width, channels), dtype=dtype, device=device)
            self.src = torch.as_tensor(stage_sources(height, self.world, block), dtype=torch.long, device=device)
            self.frame = torch.empty((height, width, channels), dtype=dtype, device=device)

    def acquire(self):
        i = self.k % self.depth
        return i, self.tiles[i], self.pending[i]

    def submit(self, i):
        ops = _post_transfer(self.tiles[i], self.stage, self.height, self.block, self.dst, self.group)
        pend = _Pending(ops, per_stream=self.tiles[i].is_cuda)
        if self.rank == self.dst:  # the current stream waits for the receives, then places the runs
            pend.wait()
            torch.index_select(self.stage, 0, self.src, out=self.frame)
            # the root's own tile reaches the stage by a copy on the current stream, which no transfer operation
            # covers: an event after it lets the renderer of frame k + depth (acquire's `prev`) wait for that read
            if self.tiles[i].is_cuda:
                pend.event = torch.cuda.Event()
                pend.event.record()
        self.pending[i] = pend
        self.k += 1

    def drain(self):
        for w in self.pending:
            if w is not None:
                w.wait()


class _Pending:
    """The operations of one frame's transfer, waited on together, and (on the root of a GPU pipeline) the event
    recorded after the local reads of the tile.  On GPU tensors wait() orders the *current* stream after them and may
    be called on several streams (an NCCL wait is a per-stream wait), so the operations are kept; on CPU tensors (gloo)
    a wait blocks the host until the operation is done and gloo must not wait for a send twice (a second waitSend
    waits for a send that never comes), so they are dropped once waited."""

    def __init__(self, ops, per_stream=False):
        self.ops = ops
        self.per_stream = per_stream
        self.event = None

    def wait(self):
        for op in self.ops:
            op.wait()
        if not self.per_stream:
            self.ops = []
        if self.event is not None:
            self.event.wait()

"""Multi-GPU tiling: one process per GPU, row-interleaved tiles, one gather to rank 0.

Pixels are independent (camera.rs:110-118 renders them in any order), so rank r renders the output
rows {y : (y // block) % N == r} (interleaved blocks balance sky/floor cost) and one collective
(torch.distributed.gather; backend "nccl" is RCCL over xGMI on ROCm, "gloo" on CPU tests) brings
the tiles to rank 0, which scatters the rows back into frame order.
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

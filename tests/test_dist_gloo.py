"""world_size-2/3 gloo tests of the multi-GPU path's host logic on CPU: the row partition, the unpadded tiles
sent to rank 0 one per part and received back to back into the staging buffer at rr_stage_row_offset (multi.cpp's
per-part ncclSend / ncclRecv layout), and the library's run placement (rr_unshuffle_host, the rows multi.cpp's
placement kernels move) reassemble a frame bit-identical to the single-process render, in f64 like the product's
tiles.  The tiles are rendered by the oracle here (test stand-in for the GPU; the GPU tests test_virtual_group_*
run the same staging and placement on the device)."""
import datetime
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, block, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from oracle.scene_yaml import build_from_yaml
    from rray_amd import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a bounded rendezvous: a port lost to another process fails the test in seconds, not after the 30-min default
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    text = open(os.path.join(ROOT, "scenes", "c3_s1024_reflect.yaml")).read()
    o, cam = build_from_yaml(text, W, H, 1)
    canvas, _ = o.render(cam, max_depth=5, threads=2, band=block, band_stride=world, band_phase=rank)
    rows = rdist.tile_rows(H, rank, world, block)
    tile = torch.from_numpy(np.ascontiguousarray(canvas[rows]))
    frame = rdist.gather_frame(tile, H, block)
    if rank == 0:
        q.put(frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _pipe_worker(rank, world, port, W, H, block, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from oracle.scene_yaml import build_from_yaml
    from rray_amd import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a bounded rendezvous: a port lost to another process fails the test in seconds, not after the 30-min default
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    text = open(os.path.join(ROOT, "scenes", "c3_s1024_reflect.yaml")).read()
    o, cam = build_from_yaml(text, W, H, 1)
    canvas, _ = o.render(cam, max_depth=5, threads=2, band=block, band_stride=world, band_phase=rank)
    rows = rdist.tile_rows(H, rank, world, block)
    pipe = rdist.FramePipeline(H, W, 3, torch.float64, torch.device("cpu"), block=block)
    frames = []
    for k in range(3):  # three frames: both buffers reused once
        i, tile, prev = pipe.acquire()
        if prev is not None:
            prev.wait()
        tile.copy_(torch.from_numpy(canvas[rows] * (k + 1)))
        pipe.submit(i)
        if rank == 0:
            frames.append(pipe.frame.clone().numpy())
    pipe.drain()
    if rank == 0:
        q.put(frames)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_pipelined_gather(oracle_mod):
    from oracle.scene_yaml import build_from_yaml

    import rray_amd  # noqa: F401

    W, H, block, world = 20, 30, 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, W, H, block, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    text = open(os.path.join(ROOT, "scenes", "c3_s1024_reflect.yaml")).read()
    o, cam = build_from_yaml(text, W, H, 1)
    full, _ = o.render(cam, max_depth=5, threads=2)
    for k, fr in enumerate(frames):
        assert np.array_equal(fr, full * (k + 1))


@pytest.mark.parametrize("world,H,block", [(2, 36, 4), (2, 33, 4), (3, 30, 4), (3, 22, 8)])
def test_two_rank_gather_matches_single_render(oracle_mod, world, H, block):
    """(3, 22, 8): 22 rows of 8-row blocks over 3 ranks — part 2 owns no rows and sends nothing."""
    from oracle.scene_yaml import build_from_yaml

    import rray_amd  # noqa: F401  (part_rows comes from the product library)

    W = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, block, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    text = open(os.path.join(ROOT, "scenes", "c3_s1024_reflect.yaml")).read()
    o, cam = build_from_yaml(text, W, H, 1)
    full, _ = o.render(cam, max_depth=5, threads=2)
    assert np.array_equal(frame, full)


PARTITIONS = ((40, 2, 8), (40, 3, 8), (40, 8, 8), (33, 2, 4), (7, 4, 2), (1, 3, 8), (40, 3, 3), (40, 2, 1), (0, 3, 8))


def test_stage_offsets_match_part_rows():
    """rr_stage_row_offset(p) (partition.hpp's closed form, which multi.cpp's receives and placement kernels use) is
    the running sum of the parts' row counts, parts with no rows included, and part == nparts gives the height."""
    import rray_amd as R

    for H, world, block in PARTITIONS + ((2160, 8, 8), (1080, 7, 8), (17, 5, 4)):
        off = 0
        for p in range(world + 1):
            assert R.stage_row_offset(H, p, world, block) == off, (H, world, block, p)
            if p < world:
                off += len(R.part_rows(H, p, world, block))
        assert off == H
    with pytest.raises(R.RRError):
        R.stage_row_offset(40, 4, 3, 8)


def test_host_unshuffle_matches_partition():
    """rr_unshuffle_host (the runs the device placement kernels move, on the host) inverts the row partition over
    the staging layout for part counts that do not divide the height, including parts with no rows at all
    (8 parts of 5 blocks) and 3-row blocks ending in a partial run."""
    import rray_amd as R

    rng = np.random.default_rng(3)
    for H, world, block in PARTITIONS:
        W = 5
        frame = rng.standard_normal((H, W, 3))
        staged = np.full((H, W, 3), np.nan)
        off = 0
        for p in range(world):
            pr = R.part_rows(H, p, world, block)
            assert R.stage_row_offset(H, p, world, block) == off
            staged[off: off + len(pr)] = frame[pr]
            off += len(pr)
        assert off == H
        assert np.array_equal(R.unshuffle(staged, H, world, block), frame), (H, world, block)


def test_host_unshuffle_refuses_wrong_shapes():
    """rr_unshuffle_host reads height rows of W * 3 doubles: rray_amd.unshuffle refuses a buffer of any other shape
    (a short stage, a 4-channel stage, a 2-D array, the old padded layout) before the library can read past it."""
    import rray_amd as R

    H, world, block, W = 40, 3, 8, 5
    rows = len(R.part_rows(H, 0, world, block))
    ok = np.zeros((H, W, 3))
    assert R.unshuffle(ok, H, world, block).shape == (H, W, 3)
    for bad in (np.zeros((H - 1, W, 3)), np.zeros((H, W, 4)), np.zeros((H, W * 3)), np.zeros((world * rows, W, 3))):
        with pytest.raises(ValueError):
            R.unshuffle(bad, H, world, block)
    with pytest.raises(ValueError):
        R.unshuffle(ok, H, 0, block)

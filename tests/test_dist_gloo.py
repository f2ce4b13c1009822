"""world_size-2/3 gloo tests of the multi-GPU path's host logic on CPU: the row partition, the padded
tiles gathered back to back (multi.cpp's ncclGather layout) and the library's un-interleave
(rr_unshuffle_host, the index arithmetic of multi.cpp's device kernel) reassemble a frame bit-identical
to the single-process render, in f64 like the product's tiles.  The tiles are rendered by the oracle here
(test stand-in for the GPU; the GPU tests test_virtual_group_* run the same assembly on the device)."""
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
    tile = torch.zeros((rdist.max_tile_rows(H, world, block), W, 3), dtype=torch.float64)
    tile[: len(rows)] = torch.from_numpy(canvas[rows])
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
        tile.zero_()
        tile[: len(rows)] = torch.from_numpy(canvas[rows] * (k + 1))
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


@pytest.mark.parametrize("world,H", [(2, 36), (2, 33), (3, 30)])
def test_two_rank_gather_matches_single_render(oracle_mod, world, H):
    from oracle.scene_yaml import build_from_yaml

    import rray_amd  # noqa: F401  (part_rows comes from the product library)

    W, block = 24, 4
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


def test_host_unshuffle_matches_partition():
    """rr_unshuffle_host (the device kernel's index arithmetic on the host) inverts the row partition for
    part counts that do not divide the height, including parts with no rows at all (8 parts of 5 blocks)."""
    import rray_amd as R

    rng = np.random.default_rng(3)
    for H, world, block in ((40, 2, 8), (40, 3, 8), (40, 8, 8), (33, 2, 4), (7, 4, 2), (1, 3, 8)):
        W = 5
        frame = rng.standard_normal((H, W, 3))
        rows = len(R.part_rows(H, 0, world, block))
        gathered = np.full((world * rows, W, 3), np.nan)
        for p in range(world):
            pr = R.part_rows(H, p, world, block)
            assert len(pr) <= rows
            gathered[p * rows: p * rows + len(pr)] = frame[pr]
        assert np.array_equal(R.unshuffle(gathered, H, world, block), frame), (H, world, block)


def test_host_unshuffle_refuses_wrong_shapes():
    """rr_unshuffle_host reads nparts * tile_rows rows of W * 3 doubles: rray_amd.unshuffle refuses a buffer
    of any other shape (a short tile, a 4-channel tile, a 2-D array) before the library can read past it."""
    import rray_amd as R

    H, world, block, W = 40, 3, 8, 5
    rows = len(R.part_rows(H, 0, world, block))
    ok = np.zeros((world * rows, W, 3))
    assert R.unshuffle(ok, H, world, block).shape == (H, W, 3)
    for bad in (np.zeros((world * rows - 1, W, 3)), np.zeros((world * rows, W, 4)), np.zeros((world * rows, W * 3)),
                np.zeros((world * (rows + 1), W, 3))):
        with pytest.raises(ValueError):
            R.unshuffle(bad, H, world, block)
    with pytest.raises(ValueError):
        R.unshuffle(ok, H, 0, block)

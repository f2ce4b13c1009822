"""GPU tests of the multi-device contexts (rr_create_multi / rr_create_rank: row tiles sent to rank 0 one per part,
received into a staging buffer and placed into frame order) and of the drop-in CLI end to end
(main.rs:49-77 -> PNG on disk).

The GPU box has one MI355X, so the RCCL groups here have one device / one rank: they exercise the whole
path through the C ABI (tile render, one RCCL group with the part's ncclSend to itself and rank 0's ncclRecv into
the staging buffer, the placement kernel, double-buffered pipelining).  The N > 1 frame assembly runs through
virtual groups (rr_create_virtual): N parts on the one device, each with its own context and streams, every
tile copied into its staging rows at rr_stage_row_offset and placed by the same per-part kernels with nparts = N —
everything of the N > 1 path except the ncclSend / ncclRecv pairs between devices.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")
CLI = os.path.join(ROOT, "rray_amd", "bin", "rray")


@pytest.fixture(scope="module")
def R():
    import rray_amd

    if rray_amd.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")
    return rray_amd


@pytest.fixture(scope="module")
def single(R):
    r = R.Renderer(0)
    yield r
    r.close()


def _scene(R, name, W, H, aa):
    text = open(os.path.join(SCENES, name)).read()
    return R.YamlScene(text, W, H, aa, obj_root=SCENES)


@pytest.mark.parametrize("kind", ["multi", "rank"])
def test_group_context_matches_single_device(R, single, kind):
    """A 1-device group (ncclCommInitAll) and a 1-rank group (ncclCommInitRank from
    rr_rccl_unique_id) render the same image as the plain context, bit for bit."""
    scene = _scene(R, "c3_s1024_reflect.yaml", 48, 40, 2)
    single.upload(scene)
    ref = single.render(scene.camera, aa=2)
    g = R.Renderer.multi([0]) if kind == "multi" else R.Renderer.rank(0, 1, 0, R.rccl_unique_id())
    try:
        assert g.info() == (1, 0, 1)
        g.upload(scene)
        got = g.render(scene.camera, aa=2)
        assert np.array_equal(got["avg"], ref["avg"])
        for k in ("rays", "shadow_rays", "shade_events"):
            assert got["stats"][k] == ref["stats"][k], k
    finally:
        g.close()


@pytest.mark.parametrize("interleave", [False, True])
@pytest.mark.parametrize("nparts,block", [(2, 8), (3, 8), (8, 8), (3, 3), (2, 1)])
def test_virtual_group_assembles_the_frame(R, single, nparts, block, interleave):
    """N virtual ranks reassemble the 1-part image bit for bit, in both partitions: cost-balanced bands (the default:
    each part's band copied into its frame rows) and interleaved row tiles (RR_PART_INTERLEAVE: each tile's runs placed
    into their frame rows with nparts = N).  40 output rows = 5 blocks of 8: not a multiple of 8N for any N here, so
    parts own different row counts, and at N = 8 three parts own no rows at all (bands: aligned to 8 rows, so at
    most 5 parts own rows); 3-row blocks end in a partial run.  C3's scene (reflection chains, depth 5) at its own
    AA."""
    W, H, aa = 48, 40, 3
    scene = _scene(R, "c3_s1024_reflect.yaml", W, H, aa)
    single.upload(scene)
    ref = single.render(scene.camera, aa=aa)
    g = R.Renderer.virtual(0, nparts)
    try:
        assert g.info() == (nparts, 0, nparts)
        g.upload(scene)
        got = g.render(scene.camera, aa=aa, block_rows=block, interleave=interleave)
        assert np.array_equal(got["avg"], ref["avg"])
        for k in ("rays", "shadow_rays", "shade_events", "samples"):
            assert got["stats"][k] == ref["stats"][k], k
        b = g.bands()
        if interleave:
            assert b is None
        else:  # calibrated: 0 .. H, non-decreasing, inner bounds on 8-row boundaries
            assert b[0] == 0 and b[-1] == H and len(b) == nparts + 1
            assert all(x <= y for x, y in zip(b, b[1:])) and all(x % 8 == 0 for x in b[:-1])
    finally:
        g.close()


@pytest.mark.parametrize("bounds", [[0, 0, 16, 40], [0, 8, 8, 40], [0, 40, 40, 40], [0, 13, 27, 40]])
def test_virtual_group_imposed_bands(R, single, bounds):
    """rr_group_set_bands: any non-decreasing bounds (empty bands, rank 0 without rows, unaligned bounds) give the
    1-part image bit for bit through the band transfer, for three frames (both tile buffers and render contexts)."""
    W, H, aa = 48, 40, 2
    scene = _scene(R, "c3_s1024_reflect.yaml", W, H, aa)
    single.upload(scene)
    ref = single.render(scene.camera, aa=aa)
    g = R.Renderer.virtual(0, 3)
    try:
        g.upload(scene)
        g.set_bands(bounds)
        for _ in range(3):
            got = g.render(scene.camera, aa=aa)
            assert np.array_equal(got["avg"], ref["avg"])
        assert g.bands() == bounds
        with pytest.raises(R.RRError):
            g.set_bands([0, 20, 10, 40])  # decreasing
    finally:
        g.close()


@pytest.mark.parametrize("name,W,H,aa,band", [("c3_s1024_reflect.yaml", 48, 40, 3, (8, 24)),  # pixel waves
                                              ("c3_s1024_reflect.yaml", 48, 40, 3, (5, 18)),
                                              ("c4_teapot.yaml", 64, 40, 2, (16, 32)),  # in-wave AA
                                              ("c4_teapot.yaml", 64, 40, 2, (3, 29)),  # partial tiles
                                              ("c5_area_light.yaml", 40, 24, 2, (8, 16)),  # jitter keyed by frame rows
                                              ("c1_readme.yaml", 48, 32, 2, (0, 8)),  # tree kernel
                                              ("c2_s1024.yaml", 64, 36, 1, (35, 36))])
def test_band_render_equals_frame_rows(R, single, name, W, H, aa, band):
    """rr_render_opts row_begin / row_end (ABI 10): a band is those rows of the whole frame bit for bit — camera rays,
    area-light jitter (keyed by the frame's sample id), recursion counters per row."""
    scene = _scene(R, name, W, H, aa)
    single.upload(scene)
    ref = single.render(scene.camera, aa=aa, canvas=True)
    got = single.render(scene.camera, aa=aa, band=band, canvas=True)
    y0, y1 = band
    assert got["avg"].shape == (y1 - y0, W, 3)
    assert np.array_equal(got["avg"], ref["avg"][y0:y1])
    assert np.array_equal(got["canvas"], ref["canvas"][y0 * aa:y1 * aa])
    assert got["stats"]["samples"] == (y1 - y0) * W * aa * aa
    with pytest.raises(R.RRError):
        single.render(scene.camera, aa=aa, band=(y1, y0))


@pytest.mark.parametrize("block", [1, 3, 8, 0])
def test_rccl_group_receives_runs_in_frame_order(R, single, block):
    """The 1-device RCCL group at several block sizes (RR_PART_INTERLEAVE; 40 output rows as 40, 14 or 5 runs of 1, 3
    or 8 rows, the last 3-row run partial): the part's tile goes to rank 0 in one ncclSend to itself, is received into
    the staging buffer and placed into its frame rows, bit for bit the plain context's image.  block 0: the band
    partition (one band: rank 0's own tile copied into the frame, no RCCL operation)."""
    scene = _scene(R, "c3_s1024_reflect.yaml", 48, 40, 1)
    single.upload(scene)
    ref = single.render(scene.camera, aa=1)
    g = R.Renderer.multi([0])
    try:
        g.upload(scene)
        for _ in range(2):  # the second frame renders into the other tile buffer and context
            got = g.render(scene.camera, aa=1, block_rows=block or 8, interleave=block != 0)
            assert np.array_equal(got["avg"], ref["avg"])
    finally:
        g.close()


def test_virtual_group_pipelined_frames(R, single):
    """rr_render_gather_device on 3 virtual ranks: three frames from two cameras enqueued back to back
    (double-buffered tiles) land in their own buffers unchanged."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    W, H, aa = 64, 44, 2
    scene = _scene(R, "c3_s1024_reflect.yaml", W, H, aa)
    cam_a = scene.camera
    cam_b = R.camera(cam_a.hsize, cam_a.vsize, cam_a.field_of_view * 0.75, list(cam_a.transform))
    single.upload(scene)
    refs = [single.render(c, aa=aa)["avg"] for c in (cam_a, cam_b)]
    g = R.Renderer.virtual(0, 3)
    bufs = []
    try:
        g.upload(scene)
        nbytes = refs[0].size * 8
        for _ in range(3):
            d = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(nbytes)) == 0
            bufs.append(d)
        opts = R._lib.RenderOpts(aa, 5, 0, 0, 0, 1, 8, R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
        for cam, d in zip((cam_a, cam_b, cam_a), bufs):
            g.render_gather_device(cam, opts, d.value, None)
        assert hip.hipDeviceSynchronize() == 0
        outs = []
        for d in bufs:
            out = np.empty_like(refs[0])
            assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_size_t(nbytes), 2) == 0
            outs.append(out)
    finally:
        for d in bufs:
            hip.hipFree(d)
        g.close()
    assert np.array_equal(outs[0], refs[0])
    assert np.array_equal(outs[1], refs[1])
    assert np.array_equal(outs[2], refs[0])


def test_group_rejects_part_and_canvas(R):
    scene = _scene(R, "c2_s1024.yaml", 32, 16, 1)
    g = R.Renderer.multi([0])
    try:
        g.upload(scene)
        with pytest.raises(R.RRError) as e:
            g.render(scene.camera, aa=1, canvas=True)
        assert e.value.code == -1
        with pytest.raises(R.RRError) as e:
            g.render(scene.camera, aa=1, part=0, nparts=2)
        assert e.value.code == -1
        with pytest.raises(R.RRError) as e:  # a group has no single-device entry point
            g.render_device(scene.camera, R._lib.RenderOpts(1, 5, 0, 0, 0, 1, 8, R._lib.RR_OUT_AVG), None, 1, None)
        assert e.value.code == -1
    finally:
        g.close()
    with pytest.raises(R.RRError):
        R.Renderer.multi([0, 0])  # distinct devices only


def test_pipelined_gathers_keep_frames_apart(R, single):
    """rr_render_gather_device is asynchronous and double-buffers its tiles: three frames from two
    cameras enqueued back to back land in their own buffers unchanged."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    W, H, aa = 64, 48, 2
    scene = _scene(R, "c3_s1024_reflect.yaml", W, H, aa)
    cam_a = scene.camera
    cam_b = R.camera(cam_a.hsize, cam_a.vsize, cam_a.field_of_view * 0.75, list(cam_a.transform))
    single.upload(scene)
    ref_a = single.render(cam_a, aa=aa)["avg"]
    ref_b = single.render(cam_b, aa=aa)["avg"]
    assert not np.array_equal(ref_a, ref_b)
    g = R.Renderer.rank(0, 1, 0, R.rccl_unique_id())
    bufs = []
    try:
        g.upload(scene)
        nbytes = ref_a.size * 8
        for _ in range(3):
            d = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(nbytes)) == 0
            bufs.append(d)
        opts = R._lib.RenderOpts(aa, 5, 0, 0, 0, 1, 8, R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
        for cam, d in zip((cam_a, cam_b, cam_a), bufs):
            g.render_gather_device(cam, opts, d.value, None)
        assert hip.hipDeviceSynchronize() == 0
        outs = []
        for d in bufs:
            out = np.empty_like(ref_a)
            assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_size_t(nbytes), 2) == 0
            outs.append(out)
    finally:
        for d in bufs:
            hip.hipFree(d)
        g.close()
    assert np.array_equal(outs[0], ref_a)
    assert np.array_equal(outs[1], ref_b)
    assert np.array_equal(outs[2], ref_a)


def _png(path):
    PIL = pytest.importorskip("PIL.Image")
    return np.asarray(PIL.open(path).convert("RGB"))


@pytest.mark.parametrize("yaml,png,aa,cwd", [
    ("objects_cube.yaml", "png/objects_cube.png", 3, GOLDEN),
    ("example1.yaml", "example1/example1.png", 3, os.path.join(GOLDEN, "example1")),
])
def test_cli_renders_reference_png(tmp_path, yaml, png, aa, cwd):
    """`rray -W 800 -H 400 -s <scene> -o out.png -a 3` (main.rs:49-77 -> render_scene_from_file,
    scene_builder_yaml.rs:429-436): the PNG written to disk equals the reference renderer's own."""
    out = tmp_path / "out.png"
    r = subprocess.run([CLI, "-W", "800", "-H", "400", "-s", yaml, "-o", str(out), "-a", str(aa)], cwd=cwd,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got, ref = _png(out), _png(os.path.join(GOLDEN, png))
    diff = int((got != ref).any(axis=2).sum())
    print(f"CLI {yaml}: {diff} of {ref.shape[0] * ref.shape[1]} pixels differ")
    assert diff == 0


def test_cli_multi_device_env(tmp_path):
    """RRAY_DEVICES selects a multi-device context in the CLI (here: the one device of the box)."""
    out1, out2 = tmp_path / "a.png", tmp_path / "b.png"
    args = ["-W", "200", "-H", "100", "-s", "objects_cone.yaml", "-a", "2"]
    r1 = subprocess.run([CLI] + args + ["-o", str(out1)], cwd=GOLDEN, capture_output=True, text=True, timeout=120)
    env = dict(os.environ, RRAY_DEVICES="0")
    r2 = subprocess.run([CLI] + args + ["-o", str(out2)], cwd=GOLDEN, capture_output=True, text=True, timeout=120,
                        env=env)
    assert r1.returncode == 0 and r2.returncode == 0, (r1.stderr, r2.stderr)
    assert np.array_equal(_png(out1), _png(out2))


def test_failed_group_frame_drains_its_work(R, single, monkeypatch):
    """A group call that fails after enqueuing work (fault injection: RRAY_TEST_FAIL_AFTER_PART = 0, so part 0's
    render is in flight when part 1 fails) drains every stream before it returns the error: close() then has
    nothing left to wait for, and a context built afterwards renders the frame bit for bit (the
    round-4 teardown hang)."""
    import time

    W, H, aa = 48, 40, 3
    scene = _scene(R, "c3_s1024_reflect.yaml", W, H, aa)
    single.upload(scene)
    ref = single.render(scene.camera, aa=aa)
    monkeypatch.setenv("RRAY_TEST_FAIL_AFTER_PART", "0")
    g = R.Renderer.virtual(0, 3)
    monkeypatch.delenv("RRAY_TEST_FAIL_AFTER_PART")
    try:
        g.upload(scene)
        with pytest.raises(R.RRError) as e:
            g.render(scene.camera, aa=aa)
        assert "injected failure" in str(e.value)
    finally:
        t0 = time.perf_counter()
        g.close()
        assert time.perf_counter() - t0 < 10.0
    g = R.Renderer.virtual(0, 3)
    try:
        g.upload(scene)
        assert np.array_equal(g.render(scene.camera, aa=aa)["avg"], ref["avg"])
    finally:
        g.close()


def test_context_outlives_the_caller_stream(R):
    """A context renders on a caller's stream that the caller destroys afterwards; the context then renders on a
    second stream and is destroyed.  Neither step touches the destroyed stream (the context waits on an event of its
    own, rr_ctx::ev_out): the round-4 teardown hang came from synchronising a group's destroyed render stream in
    rr_destroy.  Both frames equal the context's own-stream render bit for bit."""
    import time

    hip = ctypes.CDLL("libamdhip64.so.7")
    scene = _scene(R, "c3_s1024_reflect.yaml", 48, 40, 3)
    r = R.Renderer(0)
    d = ctypes.c_void_p()
    try:
        r.upload(scene)
        ref = r.render(scene.camera, aa=3)["avg"]
        nbytes = ref.size * 8
        assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(nbytes)) == 0
        opts = R._lib.RenderOpts(3, 5, 0, 0, 0, 1, 8, R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
        for _ in range(2):  # stream 1, destroyed; then stream 2, destroyed before the context
            st = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(st)) == 0
            r.render_device(scene.camera, opts, None, d.value, st.value)
            assert hip.hipStreamSynchronize(st) == 0
            out = np.empty_like(ref)
            assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_size_t(nbytes), 2) == 0
            assert np.array_equal(out, ref)
            assert hip.hipStreamDestroy(st) == 0
    finally:
        t0 = time.perf_counter()
        r.close()
        assert time.perf_counter() - t0 < 10.0
        if d.value:
            hip.hipFree(d)


def test_frame_pipeline_root_copy_orders_the_renderer(R):
    """rray_amd.dist.FramePipeline on the root: its own tile reaches the stage by a copy on the current stream, which
    no transfer operation covers.  The current stream here lags the render stream by a long sleep before each
    submit, so without the event acquire() returns for the copy, the render of frame k + 2 (filling tile k mod 2 on
    the render stream) would overwrite the tile before frame k's copy read it.  Every assembled frame must hold its
    own frame's values."""
    import socket

    import torch
    import torch.distributed as dist

    from rray_amd.dist import FramePipeline

    own = not dist.is_initialized()
    if own:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        H, W = 40, 16
        pipe = FramePipeline(H, W, 3, torch.float64, torch.device("cuda:0"), block=8, depth=2)
        render = torch.cuda.Stream()
        outs = []
        for k in range(6):
            i, tile, prev = pipe.acquire()
            with torch.cuda.stream(render):
                if prev is not None:
                    prev.wait()
                tile.fill_(float(k))
            torch.cuda.current_stream().wait_stream(render)
            torch.cuda._sleep(20_000_000)  # the current stream lags: this frame's copy of the tile runs late
            pipe.submit(i)
            outs.append(pipe.frame.clone())
        torch.cuda.synchronize()
        for k, f in enumerate(outs):
            assert torch.all(f == float(k)).item(), k
    finally:
        if own:
            dist.destroy_process_group()

"""GPU edge cases against the oracle: degenerate scenes, odd canvas sizes, recursion depths, many lights.

The reference accepts all of these (scene_builder_yaml.rs builds any list of objects and lights;
Camera::render takes any hsize/vsize; color_at recurses while remaining > 0, scene.rs:281-336), so
the GPU path must render them exactly like the oracle — including the paths the benchmark configs
never reach: partial 8x8 tiles (tile_fast off), > 2 lights (the non-prelit shading path), an empty
object list and a scene without lights.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def R():
    import rray_amd

    if rray_amd.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")
    return rray_amd


@pytest.fixture(scope="module")
def renderer(R):
    r = R.Renderer(0)
    yield r
    r.close()


def _pair(R, build):
    """The same scene built twice: through the product ABI builder and through the oracle."""
    import oracle

    b, o = R.SceneBuilder(), oracle.Oracle()
    build(b, o, oracle.Oracle.mat)
    return b, o


def _cams(R, W, H, frm=(0.0, 1.5, -5.0), to=(0.0, 1.0, 0.0)):
    import oracle

    t = oracle.Oracle.mat.view_transform(frm, to, (0, 1, 0))
    return R.camera(W, H, math.pi / 3, t), oracle.Oracle.camera(W, H, math.pi / 3, t)


def _check(renderer, b, o, W, H, aa=1, depth=5, label=""):
    renderer.upload(b)
    cam, ocam = _cams(renderer_mod(), W * aa, H * aa)
    got = renderer.render(cam, aa=aa, max_depth=depth, canvas=True)
    canvas, st = o.render(ocam, max_depth=depth)
    assert got["canvas"].shape == canvas.shape, label
    err = float(np.max(np.abs(got["canvas"] - canvas))) if canvas.size else 0.0
    print(f"{label}: max|d|={err:.3g} bit-exact={float(np.mean(got['canvas'] == canvas)):.6f}")
    assert err <= TOL, label
    avg = o.aa_average(canvas, aa)
    assert float(np.max(np.abs(got["avg"] - avg))) <= TOL, label
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"], label
    assert got["stats"]["shadow_rays"] == st["shadow_rays"], label
    assert got["stats"]["shade_events"] == st["shade_events"], label
    return got


def renderer_mod():
    import rray_amd

    return rray_amd


def _floor_and_spheres(b, o, M, reflective=0.5, lights=((-10, 10, -10),)):
    for pos in lights:
        b.point_light(pos, (1, 1, 1))
        o.point_light(pos, (1, 1, 1))
    mats = [((0.1, 0.9, 0.3, 200.0, reflective, 0.0, 1.0), M.translate(0, 0, 0)),
            ((0.1, 0.7, 0.9, 50.0, 0.0, 0.0, 1.0), M.translate(1.5, 1.0, 0.5)),
            ((0.2, 0.6, 0.6, 10.0, reflective, 0.0, 1.0), M.translate(-1.5, 1.0, 1.0))]
    b.plane(transform=M.translate(0, 0, 0), material=mats[0][0])
    o.add("plane", transform=M.translate(0, 0, 0), material=mats[0][0])
    for mat, tr in mats[1:]:
        b.sphere(transform=tr, material=mat)
        o.add("sphere", transform=tr, material=mat)


def test_empty_object_list_renders_black(renderer, R):
    """`scene: []`: every camera ray misses (color_at -> black, scene.rs:281-290)."""
    def build(b, o, M):
        b.point_light((-10, 10, -10), (1, 1, 1))
        o.point_light((-10, 10, -10), (1, 1, 1))

    b, o = _pair(R, build)
    got = _check(renderer, b, o, 24, 16, aa=2, label="empty scene")
    assert not np.any(got["avg"])


def test_scene_without_lights(renderer, R):
    """No light: shade_hit's sum over lights is empty, so only reflections of black remain."""
    b, o = _pair(R, lambda b, o, M: _floor_and_spheres(b, o, M, lights=()))
    got = _check(renderer, b, o, 24, 16, label="no lights")
    assert not np.any(got["avg"])


@pytest.mark.parametrize("W,H,aa", [(1, 1, 1), (13, 7, 1), (13, 7, 2), (9, 5, 5), (50, 3, 3)])
def test_odd_canvas_sizes(renderer, R, W, H, aa):
    """Canvases whose supersampled size is not a multiple of the 8x8 sample tile (partial tiles, the
    per-lane tile mapping) and the maximum AA level of the CLI (main.rs: max 5)."""
    b, o = _pair(R, _floor_and_spheres)
    _check(renderer, b, o, W, H, aa=aa, label=f"{W}x{H} aa{aa}")


@pytest.mark.parametrize("depth", [0, 1, 2, 7])
def test_recursion_depths(renderer, R, depth):
    """max_depth 0 (no reflected_color at all), shallow and deeper than the configs' 5."""
    b, o = _pair(R, _floor_and_spheres)
    _check(renderer, b, o, 32, 18, depth=depth, label=f"depth {depth}")


def test_three_and_four_point_lights(renderer, R):
    """More than RR_PRELIT_LIGHTS (2) lights: lighting after each shadow walk from the LDS stash."""
    for lights in (((-10, 10, -10), (10, 10, -10), (0, 5, -8)),
                   ((-10, 10, -10), (10, 10, -10), (0, 5, -8), (0, 20, 0))):
        b, o = _pair(R, lambda b, o, M, L=lights: _floor_and_spheres(b, o, M, lights=L))
        _check(renderer, b, o, 32, 18, aa=2, label=f"{len(lights)} lights")


def test_light_inside_an_object(renderer, R):
    """A light inside a sphere: every point outside it is shadowed (is_shadowed, scene.rs:234-245)."""
    b, o = _pair(R, lambda b, o, M: _floor_and_spheres(b, o, M, reflective=0.0, lights=((1.5, 1.0, 0.5),)))
    _check(renderer, b, o, 32, 18, label="light inside a sphere")


def test_camera_inside_a_sphere(renderer, R):
    """Camera rays starting inside a sphere: the first entry is behind the origin (t < 0), the hit is
    the exit point, and the normal is flipped (prepare_computations `inside`)."""
    import oracle

    def build(b, o, M):
        b.point_light((0, 0.5, 0), (1, 1, 1))
        o.point_light((0, 0.5, 0), (1, 1, 1))
        mat = (0.3, 0.7, 0.5, 100.0, 0.2, 0.0, 1.0)
        b.sphere(transform=M.scale(4, 4, 4), material=mat)
        o.add("sphere", transform=M.scale(4, 4, 4), material=mat)

    b, o = _pair(R, build)
    renderer.upload(b)
    t = oracle.Oracle.mat.view_transform((0, 0, -1), (0, 0, 1), (0, 1, 0))
    cam, ocam = R.camera(24, 16, math.pi / 2, t), oracle.Oracle.camera(24, 16, math.pi / 2, t)
    got = renderer.render(cam, aa=1, max_depth=3)["avg"]
    canvas, _ = o.render(ocam, max_depth=3)
    assert float(np.max(np.abs(got - o.aa_average(canvas, 1)))) <= TOL
    assert np.all(got > 0)


def test_kernel_times_count_matches(R, renderer):
    """rr_kernel_times returns K_COUNT = len(_lib.KERNELS) kernels (trace .. chain, deep), and a reflective scene's
    frame is timed under `chain` (one launch per frame)."""
    import ctypes as C
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "scenes", "c3_s1024_reflect.yaml")).read()
    scene = R.YamlScene(text, 32, 16, 1)
    renderer.upload(scene)
    renderer.kernel_profile(True)
    try:
        renderer.render(scene.camera, aa=1)
        ms, n = (C.c_double * 16)(), (C.c_uint64 * 16)()
        k = R.lib().rr_kernel_times(renderer.h, ms, n, 16)
        assert k == len(R._lib.KERNELS)
        times = renderer.kernel_times()
        assert list(times) == R._lib.KERNELS
        assert times["chain"][1] == 1 and times["chain"][0] > 0.0
    finally:
        renderer.kernel_profile(False)

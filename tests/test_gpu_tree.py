"""GPU tests of the color_at trees of transparent scenes inside the camera wave (render_tree.inc tree_kernel,
DESIGN.md §3.13): every camera sample's reflected / refracted recursion (scene.rs:159-178, 281-290, 310-336) on a
per-lane stack, one launch per frame.

* The tree kernel and the per-level wavefront kernels (RRAY_NO_TREE=1: trace / n1n2 / shade launches per level and the
  bottom-up combine passes) give the same canvas, image and recursion counters bit for bit, on flat, group, general
  (CSG, cube / cylinder / cone) and area-light scenes, at aa 1 / 2 / 3 (plain, in-wave and pixel-wave delivery).
* Against the oracle: nested glass to every max_depth up to RR_MAX_DEPTH (8, the stack's deepest frames), a glass
  sphere under an area light (the block-synchronised area walks inside the tree loop), glass inside a group.
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")
TOL = 1e-5
COUNTS = ("rays", "shadow_rays", "shade_events", "n1n2_scans", "samples", "nan_rays")


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


def _render_with(renderer, cam, env, **kw):
    os.environ.update(env)
    try:
        return renderer.render(cam, **kw)
    finally:
        for k in env:
            del os.environ[k]


def _same(a, b, label):
    assert np.array_equal(a["avg"], b["avg"]), label + " avg"
    if a["canvas"] is not None:
        assert np.array_equal(a["canvas"], b["canvas"]), label + " canvas"
    for k in COUNTS:
        assert a["stats"][k] == b["stats"][k], (label, k, a["stats"][k], b["stats"][k])


TREE_SCENES = [  # (directory, file, W, H, aa)
    (SCENES, "c1_readme.yaml", 64, 48, 1),
    (SCENES, "c1_readme.yaml", 48, 32, 2),
    (SCENES, "c1_readme.yaml", 36, 24, 3),  # pixel waves
    (GOLDEN, "shapes_glass.yaml", 64, 32, 2),  # general kernels: cube / cylinder / cone / CSG glass
    (GOLDEN, "shapes_glass.yaml", 45, 30, 3),
    (GOLDEN, "patterns_noise_mix.yaml", 64, 32, 1),  # complex patterns (the out-of-line pattern evaluator)
    (GOLDEN, "shapes_torus.yaml", 48, 24, 2),
    (os.path.join(GOLDEN, "example1"), "example1.yaml", 80, 40, 1),
]


@pytest.mark.parametrize("d,name,W,H,aa", TREE_SCENES)
def test_tree_kernel_matches_levels(R, renderer, d, name, W, H, aa):
    text = open(os.path.join(d, name)).read()
    scene = R.YamlScene(text, W, H, aa, obj_root=d)
    renderer.upload(scene)
    canvas = aa != 3  # pixel-wave frames write the canvas too when asked, but keep one case on the pure average path
    tree = _render_with(renderer, scene.camera, {}, aa=aa, max_depth=5, seed=11, canvas=canvas)
    levels = _render_with(renderer, scene.camera, {"RRAY_NO_TREE": "1"}, aa=aa, max_depth=5, seed=11, canvas=canvas)
    _same(tree, levels, f"{name} {W}x{H} aa{aa}")
    # the tree path is the one that ran: one K_CHAIN launch, no trace / n1n2 / shade / combine launches
    renderer.kernel_profile(True)
    renderer.render(scene.camera, aa=aa, max_depth=5, seed=11)
    kt = renderer.kernel_times()
    renderer.kernel_profile(False)
    assert kt["chain"][1] == 1 and kt["combine"][1] == 0 and kt["n1n2"][1] == 0 and kt["shade"][1] == 0, kt


def _glass_pair(R, area=False, group=False):
    """Nested glass (ray.rs:196-235 geometry, a mirror-glass outer sphere) over a reflective checker floor, built
    through the product's SceneBuilder and the oracle side by side."""
    import oracle

    M = oracle.Oracle.mat
    b, o = R.SceneBuilder(), oracle.Oracle()
    if area:
        b.area_light((-3, 4, -4), (1.5, 0, 0), (0, 1.5, 0), (1, 1, 1), 3)
        o.area_light((-3, 4, -4), (1.5, 0, 0), (0, 1.5, 0), (1, 1, 1), 3)
    else:
        b.point_light((-10, 10, -10), (1, 1, 1))
        o.point_light((-10, 10, -10), (1, 1, 1))
    bp, op = -1, -1
    if group:
        g = M.translate(0.2, 0.1, 0.0)
        bp = b.group(transform=g)
        op = o.add("group", transform=g)
    for tr, ri, refl in ((M.scale(2, 2, 2), 1.5, 0.3), (M.translate(0, 0, -0.25), 2.0, 0.0),
                         (M.translate(0, 0, 0.25), 2.5, 0.5)):
        mat = (0.1, 0.9, 0.9, 200.0, refl, 0.9, ri)
        b.sphere(transform=tr, material=mat, parent=bp)
        o.add("sphere", parent=op, transform=tr, material=mat)
    fl = (0.1, 0.9, 0.9, 200.0, 0.2, 0.0, 1.0)
    b.plane(transform=M.translate(0, -2.5, 0), material=fl,
            pattern=b.pattern("checker", a=b.pattern("solid", color=(1, 1, 1)), b=b.pattern("solid", color=(0, 0, 0))))
    pa, pb = o.pattern("solid", color=(1, 1, 1)), o.pattern("solid", color=(0, 0, 0))
    o.add("plane", transform=M.translate(0, -2.5, 0), material=fl, pattern=o.pattern("checker", a=pa, b=pb))
    cam_t = M.view_transform((0.3, 1.0, -6.0), (0, 0, 0), (0, 1, 0))
    return b, o, cam_t


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 8])
@pytest.mark.parametrize("aa", [1, 2, 3])
def test_glass_tree_depths_match_oracle(R, renderer, depth, aa):
    """Every max_depth up to RR_MAX_DEPTH (the per-lane stack full) against the oracle: canvas, image, counters."""
    import oracle

    b, o, cam_t = _glass_pair(R)
    renderer.upload(b)
    W, H = 36, 24  # multiples of 1, 2 and 3
    cam = R.camera(W, H, math.pi / 3, cam_t)
    got = renderer.render(cam, aa=aa, max_depth=depth, seed=5, canvas=True)
    canvas, st = o.render(oracle.Oracle.camera(W, H, math.pi / 3, cam_t), max_depth=depth, seed=5)
    assert np.max(np.abs(got["canvas"] - canvas)) <= TOL
    ref = o.aa_average(canvas, aa)
    err = float(np.max(np.abs(got["avg"] - ref)))
    assert err <= TOL, err
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shadow_rays"] == st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]
    if depth >= 2:
        assert st["rays"] - st["shadow_rays"] > 2 * W * H  # the trees are deep here


@pytest.mark.parametrize("area,group", [(True, False), (False, True), (True, True)])
def test_glass_tree_area_light_and_groups(R, renderer, area, group):
    """The area-light tree kernels (block-synchronised shadow walks inside the tree loop, jitter keyed by each node's
    path code) and the group kernels, against the oracle and against the per-level kernels."""
    import oracle

    b, o, cam_t = _glass_pair(R, area=area, group=group)
    renderer.upload(b)
    W, H = 40, 32
    cam = R.camera(W, H, math.pi / 3, cam_t)
    got = renderer.render(cam, aa=2, max_depth=5, seed=9, canvas=True)
    canvas, st = o.render(oracle.Oracle.camera(W, H, math.pi / 3, cam_t), max_depth=5, seed=9)
    err = float(np.max(np.abs(got["canvas"] - canvas)))
    assert err <= TOL, err
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shadow_rays"] == st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]
    levels = _render_with(renderer, cam, {"RRAY_NO_TREE": "1"}, aa=2, max_depth=5, seed=9, canvas=True)
    _same(got, levels, f"glass area={area} group={group}")


def test_color_at_queries_through_the_tree(R, renderer):
    """rr_color_at (Scene::color_at for given rays) runs the tree kernel on caller rays (A.rays0): equal to the
    per-level kernels and to the oracle's color_at."""
    import oracle

    b, o, cam_t = _glass_pair(R)
    renderer.upload(b)
    rng = np.random.default_rng(3)
    n = 500
    org = np.tile([0.3, 1.0, -6.0], (n, 1)) + rng.normal(0, 0.05, (n, 3))
    d = np.array([0.0, 0.0, 0.0]) - org + rng.normal(0, 0.6, (n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    got = renderer.color_at(org, d, remaining=5)
    os.environ["RRAY_NO_TREE"] = "1"
    try:
        lev = renderer.color_at(org, d, remaining=5)
    finally:
        del os.environ["RRAY_NO_TREE"]
    assert np.array_equal(got, lev)
    ref = np.array([o.color_at(org[i], d[i], 5) for i in range(n)])
    assert np.max(np.abs(got - ref)) <= TOL

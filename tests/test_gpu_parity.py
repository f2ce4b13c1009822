"""GPU parity: the HIP render path (through the C ABI) against the CPU oracle.

Gate (north_star): every channel of the AA-averaged f64 image within 1e-5 of the oracle before u8
quantisation.  The kernels restate the reference op-for-op (no FMA contraction), so the observed
difference is expected to be 0 except where the device's pow() differs from glibc's in the last
ulp (specular term); the tests report the bit-exact fraction alongside the gate.
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
S2 = math.sqrt(2.0)


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


def _yaml_pair(name, W, H, aa, obj_root=SCENES, path=None):
    import rray_amd as R
    from oracle.scene_yaml import build_from_yaml

    text = open(path or os.path.join(SCENES, name)).read()
    return R.YamlScene(text, W, H, aa, obj_root=obj_root), build_from_yaml(text, W, H, aa, obj_root=obj_root)


def _compare(got, ref, label):
    err = float(np.max(np.abs(got - ref))) if got.size else 0.0
    exact = float(np.mean(got == ref)) if got.size else 1.0
    print(f"{label}: max|d|={err:.3g} bit-exact={exact:.6f}")
    assert np.all(np.isfinite(got)), label
    assert err <= TOL, f"{label}: max |delta| {err} > {TOL}"
    return err, exact


CASES = [  # (scene file, W, H, aa)
    ("c1_readme.yaml", 64, 48, 1),
    ("c1_readme.yaml", 32, 24, 3),
    ("c2_s1024.yaml", 64, 36, 1),
    ("c3_s1024_reflect.yaml", 48, 27, 2),
    ("c3_s1024_reflect.yaml", 32, 18, 3),  # C3's own AA
    ("c4_teapot.yaml", 48, 27, 1),
    ("c4_teapot.yaml", 48, 27, 2),  # C4's own AA
    ("c5_area_light.yaml", 40, 20, 2),
]


@pytest.mark.parametrize("name,W,H,aa", CASES)
def test_render_matches_oracle(renderer, name, W, H, aa):
    scene, (o, cam) = _yaml_pair(name, W, H, aa)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=5, seed=7, canvas=True)
    canvas, st = o.render(cam, max_depth=5, seed=7, threads=0)
    ref = o.aa_average(canvas, aa)
    _compare(got["canvas"], canvas, f"{name} {W}x{H} aa{aa} canvas")
    _compare(got["avg"], ref, f"{name} {W}x{H} aa{aa} avg")
    # counters agree with the reference's recursion structure
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shadow_rays"] == st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]


def test_cost_ordered_tiles_change_no_result(R, renderer):
    """Group scenes without secondary rays render level 0 in cost order from a layout's second frame on
    (tile_order_kernel): frames 2..4 of the C4 thumbnail, a moved camera of the same layout
    (the order is kept) and back, must equal the first, launch-order frame bit for bit, counters included."""
    import math as m

    scene, (o, cam) = _yaml_pair("c4_teapot.yaml", 64, 40, 2)
    renderer.upload(scene)
    first = renderer.render(scene.camera, aa=2, max_depth=5)
    canvas, _ = o.render(cam, max_depth=5)
    _compare(first["avg"], o.aa_average(canvas, 2), "c4 64x40 aa2 frame 1")
    for k in range(3):
        again = renderer.render(scene.camera, aa=2, max_depth=5)
        assert np.array_equal(again["avg"], first["avg"]), f"frame {k + 2}"
        drop = ("kernel_ms",)  # timing, not a count
        assert {k: v for k, v in again["stats"].items() if k not in drop} == \
            {k: v for k, v in first["stats"].items() if k not in drop}
    from oracle.oracle import Oracle

    t = list(scene.camera.transform)
    moved = R.camera(128, 80, m.pi / 3.2, t)  # same layout, another view: rendered in the first view's tile order
    mv = renderer.render(moved, aa=2, max_depth=5)
    ocam = Oracle.camera(128, 80, m.pi / 3.2, t)
    mcanvas, _ = o.render(ocam, max_depth=5)
    _compare(mv["avg"], o.aa_average(mcanvas, 2), "c4 64x40 aa2 moved camera (kept tile order)")
    ref_moved = renderer.render(moved, aa=2, max_depth=5)
    assert np.array_equal(mv["avg"], ref_moved["avg"])
    back = renderer.render(scene.camera, aa=2, max_depth=5)
    assert np.array_equal(back["avg"], first["avg"])


@pytest.mark.parametrize("name,W,H,aa", [("c4_teapot.yaml", 64, 40, 2), ("c3_s1024_reflect.yaml", 48, 24, 3)])
def test_order_units_change_no_result(renderer, monkeypatch, name, W, H, aa):
    """The cost order's unit (api.cpp run_levels) — one camera wave (the default) or a block's four adjacent tiles
    (RRAY_ORDER_GROUP=4) — changes which wave renders which tile, never a pixel: a group scene's level-0 frames and
    a chain scene's pixel-wave frames (aa 3), three under each unit (guessed order, then measured orders), are
    bit-identical to each other and within the gate of the oracle, counters equal."""
    scene, (o, cam) = _yaml_pair(name, W, H, aa)
    renderer.upload(scene)
    canvas, _ = o.render(cam, max_depth=5)
    ref = o.aa_average(canvas, aa)
    first = None
    drop = ("kernel_ms",)  # timing, not a count
    for unit in ("1", "4"):
        monkeypatch.setenv("RRAY_ORDER_GROUP", unit)
        for k in range(3):
            got = renderer.render(scene.camera, aa=aa, max_depth=5)
            if first is None:
                _compare(got["avg"], ref, f"{name} {W}x{H} aa{aa} order unit {unit}")
                first = got
                continue
            assert np.array_equal(got["avg"], first["avg"]), f"order unit {unit}, frame {k + 1}"
            assert {q: v for q, v in got["stats"].items() if q not in drop} == \
                {q: v for q, v in first["stats"].items() if q not in drop}


@pytest.mark.parametrize("name,W,H,aa", [("c4_teapot.yaml", 48, 28, 2), ("c4_teapot.yaml", 40, 24, 4),
                                         ("c2_s1024.yaml", 32, 20, 4), ("c2_s1024.yaml", 16, 10, 8),
                                         ("c1_readme.yaml", 24, 16, 2)])
def test_in_wave_aa_average(renderer, name, W, H, aa):
    """Frames without secondary rays at aa 2 / 4 / 8 with full 8x8 sample tiles: the level-0 waves box-average
    their own samples (deliver_wave_avg, canvas.rs:85-96 order) and no canvas is written.  The image must
    equal the oracle's average; with the canvas requested as well, both outputs must match.  (The README
    scene's glass sphere has secondary rays: the canvas path, for contrast.)"""
    scene, (o, cam) = _yaml_pair(name, W, H, aa)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=5, seed=7)
    canvas, st = o.render(cam, max_depth=5, seed=7, threads=0)
    ref = o.aa_average(canvas, aa)
    _compare(got["avg"], ref, f"{name} {W}x{H} aa{aa} in-wave avg")
    both = renderer.render(scene.camera, aa=aa, max_depth=5, seed=7, canvas=True)
    _compare(both["canvas"], canvas, f"{name} {W}x{H} aa{aa} canvas")
    # the wave's reduction is exactly canvas.rs's box average of the GPU's own samples
    assert np.array_equal(both["avg"], got["avg"])
    assert np.array_equal(got["avg"], o.aa_average(both["canvas"], aa))
    assert got["stats"]["shade_events"] == st["shade_events"]


def test_render_matches_committed_golden(renderer, R):
    """Committed oracle outputs (tests/golden/make_golden.py) — no live oracle needed.  Every config
    scene, C3 and C4 also at their own AA levels (3 and 2)."""
    import json

    meta = json.load(open(os.path.join(GOLDEN, "golden_renders.json")))
    assert {(g["scene"], g["aa"]) for g in meta} >= {("c3_s1024_reflect.yaml", 3), ("c4_teapot.yaml", 2)}
    for g in meta:
        scene = R.YamlScene(open(os.path.join(SCENES, g["scene"])).read(), g["W"], g["H"], g["aa"], obj_root=SCENES)
        renderer.upload(scene)
        got = renderer.render(scene.camera, aa=g["aa"], max_depth=5, seed=g["seed"])
        ref = np.load(os.path.join(GOLDEN, g["file"]))
        _compare(got["avg"], ref, "golden " + g["file"])


@pytest.mark.parametrize("name", ["checker_pattern.yaml", "stripe_pattern.yaml", "gradient_pattern.yaml",
                                  "ring_pattern.yaml", "blend_pattern.yaml", "triangle.yaml"])
def test_reference_example_scenes(renderer, name):
    scene, (o, cam) = _yaml_pair(name, 40, 20, 1, obj_root=GOLDEN, path=os.path.join(GOLDEN, name))
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=1, max_depth=5)
    canvas, _ = o.render(cam, max_depth=5)
    _compare(got["avg"], o.aa_average(canvas, 1), name)


@pytest.mark.parametrize("name,W,H,aa", [("shapes_csg.yaml", 64, 32, 2), ("shapes_glass.yaml", 64, 32, 2),
                                         ("shapes_mixed.yaml", 64, 32, 2), ("objects_cylinder.yaml", 48, 24, 1),
                                         ("objects_cone.yaml", 48, 24, 1), ("patterns_noise_mix.yaml", 64, 32, 2),
                                         ("noise_pattern.yaml", 64, 32, 1), ("perturbed_pattern.yaml", 64, 32, 1),
                                         ("objects_sphere.yaml", 48, 24, 2), ("textures_mix.yaml", 96, 48, 2),
                                         ("textures_mix.yaml", 200, 100, 1), ("shapes_torus.yaml", 96, 48, 2),
                                         ("shapes_torus.yaml", 200, 100, 1)])
def test_shape_scenes(renderer, name, W, H, aa):
    """Cube / cylinder / cone / CSG through the general kernel variant: 4-entry
    leaves, CSG subtrees evaluated per lane, n1/n2 over filtered entries.  Perturbed / noise
    patterns (next-3): the f32 Perlin lattice restated op-for-op, nested in other patterns.  Image
    textures (next-3): uv_mapping per shape kind + texel fetch from the decoded PNGs."""
    scene, (o, cam) = _yaml_pair(name, W, H, aa, obj_root=GOLDEN, path=os.path.join(GOLDEN, name))
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=5, canvas=True)
    canvas, st = o.render(cam, max_depth=5)
    _compare(got["canvas"], canvas, name + " canvas")
    _, exact = _compare(got["avg"], o.aa_average(canvas, aa), name + " avg")
    # regression guard on the bit-exact fraction: only libm's last ulp may differ (pow; the torus solver's
    # transcendentals round like glibc since round 4, DESIGN.md §3.8 — measured 1.000000 on both torus cases)
    assert exact >= 0.999, f"{name}: bit-exact fraction {exact:.6f}"
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shadow_rays"] == st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]


MIRRORS = """camera:
  fov: 1.0
  from: [0, 1, -4.5]
  to: [0.3, 0.9, 4]
  up: [0, 1, 0]
lights:
  - type: point
    color: [1, 1, 1]
    position: [0, 3, -3]
scene:
  - type: plane
    transforms:
      - type: rotate
        axis: z
        angle: 90
      - type: translate
        amount: [-1.5, 0, 0]
    material:
      pattern:
        type: solid
        color: [0.2, 0.3, 0.4]
      specular: 0.3
      reflective: 0.9
  - type: plane
    transforms:
      - type: rotate
        axis: z
        angle: 90
      - type: translate
        amount: [1.5, 0, 0]
    material:
      pattern:
        type: solid
        color: [0.4, 0.3, 0.2]
      reflective: 0.8
  - type: plane
    transforms: []
    material:
      pattern:
        type: checker
        pattern_a:
          type: solid
          color: [0.9, 0.9, 0.9]
        pattern_b:
          type: solid
          color: [0.1, 0.1, 0.1]
      reflective: 0.25
  - type: sphere
    transforms:
      - type: translate
        amount: [0.4, 0.8, 2]
    material:
      pattern:
        type: solid
        color: [0.8, 0.1, 0.1]
      specular: 0.9
      shininess: 50
      reflective: 0.5
"""


@pytest.mark.parametrize("name,W,H,aa", [("c3_s1024_reflect.yaml", 32, 18, 3), ("c3_s1024_reflect.yaml", 48, 27, 2),
                                         ("c3_s1024_reflect.yaml", 64, 36, 1), ("c5_area_light.yaml", 40, 20, 2),
                                         ("c1_readme.yaml", 32, 24, 2)])
def test_reflection_chains_in_kernel_match_levels(renderer, name, W, H, aa):
    """Scenes without transparency run every reflection chain inside its camera wave (chain_kernel,
    DESIGN.md §3); RRAY_NO_CHAIN=1 selects the per-level wavefront kernels (HBM event queues, one launch per
    depth).  Both must give the same canvas, image and counters bit for bit (the README scene has a glass
    sphere: unfused levels either way)."""
    scene, _ = _yaml_pair(name, W, H, aa)
    renderer.upload(scene)

    def render_with(env):
        os.environ.update(env)
        try:
            return renderer.render(scene.camera, aa=aa, max_depth=5, seed=3, canvas=True)
        finally:
            for k in env:
                del os.environ[k]

    chain = render_with({})
    # timing and the walks' work counts (culling differs between the kernels' walk variants)
    drop = ("kernel_ms", "exact_flops", "wave_visits", "prim_tests", "group_tests", "group_hits")
    # RRAY_DEEP=1: chains still reflecting at depth 2 finish in the deep-queue launch (frames without in-wave AA)
    for env in ({"RRAY_NO_CHAIN": "1"}, {"RRAY_DEEP": "1"}):
        other = render_with(env)
        assert np.array_equal(chain["canvas"], other["canvas"]), (name, env)
        assert np.array_equal(chain["avg"], other["avg"]), (name, env)
        assert {k: v for k, v in chain["stats"].items() if k not in drop} == \
            {k: v for k, v in other["stats"].items() if k not in drop}, (name, env)


@pytest.mark.parametrize("depth", [0, 1, 2, 3, 5, 8])
@pytest.mark.parametrize("aa", [1, 2, 3])
def test_mirror_corridor_depths(R, renderer, depth, aa):
    """Two facing mirrors and a reflective floor: chains run to every max_depth up to RR_MAX_DEPTH (8), the
    in-kernel stack's deepest records included, against the oracle (canvas, image, counters)."""
    from oracle.scene_yaml import build_from_yaml

    W, H = 40, 24
    scene = R.YamlScene(MIRRORS, W, H, aa)
    o, cam = build_from_yaml(MIRRORS, W, H, aa)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=depth, canvas=True)
    os.environ["RRAY_DEEP"] = "1"  # the deep-queue launch too (aa 1 and 3: samples delivered one by one)
    try:
        deep = renderer.render(scene.camera, aa=aa, max_depth=depth, canvas=True)
    finally:
        del os.environ["RRAY_DEEP"]
    assert np.array_equal(deep["canvas"], got["canvas"]) and np.array_equal(deep["avg"], got["avg"])
    canvas, st = o.render(cam, max_depth=depth)
    _compare(got["canvas"], canvas, f"mirrors aa{aa} depth {depth} canvas")
    _compare(got["avg"], o.aa_average(canvas, aa), f"mirrors aa{aa} depth {depth} avg")
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shadow_rays"] == st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]
    if depth >= 5:  # the corridor really recurses that deep
        assert st["rays"] - st["shadow_rays"] > 3 * W * H * aa * aa


@pytest.mark.parametrize("W,H", [(37, 13), (8, 1), (7, 2), (50, 9)])
def test_pixel_waves_odd_sizes(R, renderer, W, H):
    """aa = 3 frames with reflection chains average in the wave (pixel waves: 7 whole pixels per wave, bands of two
    output rows, render_common.inc pixel_wave): widths that leave a band's last wave short, odd row counts (a
    one-row last band), one-row frames — canvas, image and counters against the oracle, and the image against the
    aa_kernel path (RRAY_NO_PW=1) bit for bit."""
    from oracle.scene_yaml import build_from_yaml

    scene = R.YamlScene(MIRRORS, W, H, 3)
    o, cam = build_from_yaml(MIRRORS, W, H, 3)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=3, max_depth=5)
    both = renderer.render(scene.camera, aa=3, max_depth=5, canvas=True)
    canvas, st = o.render(cam, max_depth=5)
    _compare(both["canvas"], canvas, f"mirrors {W}x{H} aa3 canvas")
    _compare(got["avg"], o.aa_average(canvas, 3), f"mirrors {W}x{H} aa3 pixel waves")
    assert np.array_equal(got["avg"], both["avg"])
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]
    os.environ["RRAY_NO_PW"] = "1"
    try:
        ref = renderer.render(scene.camera, aa=3, max_depth=5)
    finally:
        del os.environ["RRAY_NO_PW"]
    assert np.array_equal(got["avg"], ref["avg"])


@pytest.mark.parametrize("W,H,aa", [(160, 80, 2), (400, 200, 1)])
def test_torus_jpeg_texture_scene(renderer, W, H, aa):
    """The reference's examples/objects/torus.yaml: a torus with the JPEG texture
    examples/Texturelabs_Stone_138M.jpg (texture.rs:15-19), decoded by the product front-end
    (jpeg.cpp) and by PIL in the oracle.  The texels are bit-identical (tests/test_jpeg.py), and the torus
    solver's transcendentals round like the host glibc (host_libm.inc), so the frames are
    bit-exact (measured 1.000000, round 4); held to the north_star tolerance like every scene, with equal
    recursion counters."""
    root = os.path.join(GOLDEN, "example1")
    scene, (o, cam) = _yaml_pair("torus.yaml", W, H, aa, obj_root=root, path=os.path.join(root, "torus.yaml"))
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=5, canvas=True)
    canvas, st = o.render(cam, max_depth=5)
    _, exact_c = _compare(got["canvas"], canvas, "torus.yaml canvas")
    _, exact = _compare(got["avg"], o.aa_average(canvas, aa), "torus.yaml avg")
    # regression guard: glibc-rounded transcendentals leave at most glibc's rare last-ulp misses
    assert exact_c >= 0.999 and exact >= 0.999, f"torus.yaml: bit-exact fractions {exact_c:.4f} / {exact:.4f}"
    assert got["stats"]["rays"] == st["rays"] - st["shadow_rays"]
    assert got["stats"]["shade_events"] == st["shade_events"]


@pytest.mark.parametrize("name,png,aa", [("objects_cylinder.yaml", "objects_cylinder.png", 3),
                                         ("objects_cone.yaml", "objects_cone.png", 3),
                                         ("objects_sphere.yaml", "objects_sphere.png", 3),
                                         ("objects_cube.yaml", "objects_cube.png", 3),
                                         ("noise_pattern.yaml", "noise_pattern.png", 1),
                                         ("perturbed_pattern.yaml", "perturbed_pattern.png", 1)])
def test_reference_png_through_gpu(renderer, R, name, png, aa):
    """The reference renderer's own 800x400 outputs (examples/objects/*.png at aa=3,
    examples/patterns/*.png at aa=1), reproduced by the GPU path through quantisation
    (canvas.rs:76-105)."""
    PIL = pytest.importorskip("PIL.Image")
    text = open(os.path.join(GOLDEN, name)).read()
    scene = R.YamlScene(text, 800, 400, aa, obj_root=GOLDEN)
    renderer.upload(scene)
    avg = renderer.render(scene.camera, aa=aa, max_depth=5)["avg"]
    q = R.quantize(avg)[..., :3]
    ref = np.asarray(PIL.open(os.path.join(GOLDEN, "png", png)).convert("RGB"))
    diff = int((q != ref).any(axis=2).sum())
    print(f"{png}: {diff} of {ref.shape[0] * ref.shape[1]} pixels differ")
    assert diff == 0


def test_c1_readme_test1_png_through_gpu(renderer, R):
    """C1 pinned to the reference's own image: examples/test1.png is the README scene (README.md:106-113,
    `rray -W 800 -H 400`, aa=1).  The glass sphere exercises reflect + refract + Schlick + n1/n2."""
    PIL = pytest.importorskip("PIL.Image")
    text = open(os.path.join(SCENES, "c1_readme.yaml")).read()
    scene = R.YamlScene(text, 800, 400, 1, obj_root=SCENES)
    renderer.upload(scene)
    avg = renderer.render(scene.camera, aa=1, max_depth=5)["avg"]
    q = R.quantize(avg)[..., :3]
    ref = np.asarray(PIL.open(os.path.join(GOLDEN, "png", "test1.png")).convert("RGB"))
    diff = int((q != ref).any(axis=2).sum())
    print(f"test1.png: {diff} of {ref.shape[0] * ref.shape[1]} pixels differ")
    assert diff == 0


def test_c1_config_full_frame(renderer):
    """BASELINE configs[0]: the README scene at 800x600 aa=1, whole frame against the oracle."""
    scene, (o, cam) = _yaml_pair("c1_readme.yaml", 800, 600, 1)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=1, max_depth=5)
    canvas, st = o.render(cam, max_depth=5, threads=0)
    _compare(got["avg"], o.aa_average(canvas, 1), "c1 800x600 aa1")
    assert got["stats"]["shade_events"] == st["shade_events"]


def test_example1_png_through_gpu(renderer, R):
    """The reference's headline image (README example1.png, 800x400, aa=3): torus (roots 0.0.8
    quartic), earthmap texture, noise / perturbed, CSG, cube / cylinder / cone, the full teapot."""
    PIL = pytest.importorskip("PIL.Image")
    root = os.path.join(GOLDEN, "example1")
    text = open(os.path.join(root, "example1.yaml")).read()
    scene = R.YamlScene(text, 800, 400, 3, obj_root=root)
    renderer.upload(scene)
    avg = renderer.render(scene.camera, aa=3, max_depth=5)["avg"]
    q = R.quantize(avg)[..., :3]
    ref = np.asarray(PIL.open(os.path.join(root, "example1.png")).convert("RGB"))
    diff = int((q != ref).any(axis=2).sum())
    print(f"example1.png: {diff} of {ref.shape[0] * ref.shape[1]} pixels differ")
    assert diff == 0


def test_noise_zero_octaves_is_nan(renderer, R):
    """octave_perlin with 0 octaves returns 0/0 (noise.rs:11-29): the noise pattern's colour is NaN
    (b * NaN), which quantises to 0 (canvas.rs `as u8`).  Both sides must agree NaN-for-NaN."""
    from oracle.scene_yaml import build_from_yaml

    text = ("camera: {fov: 60, from: [0, 1.5, -5], to: [0, 1, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [-10, 10, -10]\nscene:\n  - type: plane\n  - type: sphere\n"
            "    transforms: [{type: translate, amount: [0, 1, 0]}]\n    material:\n      pattern:\n"
            "        type: noise\n        octaves: 0\n        color_a: [1, 0, 0]\n        color_b: [0, 0, 1]\n")
    scene = R.YamlScene(text, 32, 16, 1)
    o, cam = build_from_yaml(text, 32, 16, 1)
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=1, max_depth=5)["avg"]
    canvas, _ = o.render(cam, max_depth=5)
    ref = o.aa_average(canvas, 1)
    assert np.isnan(ref).any() and np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got, ref, equal_nan=True)
    assert np.array_equal(R.quantize(got), o.quantize(ref))


def test_multi_part_tiles_are_bit_identical(renderer, R):
    """Row-interleaved tiles (the multi-GPU partition) reassemble to the 1-part image bit-for-bit."""
    scene, _ = _yaml_pair("c3_s1024_reflect.yaml", 48, 40, 1)
    renderer.upload(scene)
    full = renderer.render(scene.camera, aa=1)["avg"]
    for nparts in (2, 3, 8):
        img = np.zeros_like(full)
        for p in range(nparts):
            rows = R.part_rows(40, p, nparts, 4)
            img[rows] = renderer.render(scene.camera, aa=1, part=p, nparts=nparts, block_rows=4)["avg"]
        assert np.array_equal(img, full), nparts


def test_batched_passes_are_bit_identical(renderer, R):
    """A frame split into many wavefront passes (RRAY_BATCH) renders the same image as one pass."""
    scene, _ = _yaml_pair("c3_s1024_reflect.yaml", 48, 27, 2)
    renderer.upload(scene)
    one = renderer.render(scene.camera, aa=2, canvas=True)
    os.environ["RRAY_BATCH"] = "1024"
    try:
        small = R.Renderer(0)
    finally:
        del os.environ["RRAY_BATCH"]
    try:
        small.upload(scene)
        many = small.render(scene.camera, aa=2, canvas=True)  # 96x54 samples -> 6 passes
    finally:
        small.close()
    assert np.array_equal(one["canvas"], many["canvas"])
    assert np.array_equal(one["avg"], many["avg"])
    assert one["stats"]["rays"] == many["stats"]["rays"]


# ---------------------------------------------------------------- known-answer tests through the GPU
def default_scene(R, O=None):
    """scene.rs:79-92 on both sides."""
    b = R.SceneBuilder()
    b.point_light((-10, 10, -10), (1, 1, 1))
    p = b.pattern("solid", color=(0.8, 1.0, 0.6))
    b.sphere(material=(0.1, 0.7, 0.2, 200.0, 0.0, 0.0, 1.0), pattern=p)
    b.sphere(transform=(0.5, 0, 0, 0, 0, 0.5, 0, 0, 0, 0, 0.5, 0, 0, 0, 0, 1))
    return b


def test_color_at_known_answers(renderer, R):  # scene.rs:454-468, 610-629
    renderer.upload(default_scene(R))
    c = renderer.color_at([(0, 0, -5), (0, 0, -5)], [(0, 1, 0), (0, 0, 1)], remaining=5)
    assert np.array_equal(c[0], [0, 0, 0])
    assert np.allclose(c[1], [0.38066, 0.47583, 0.2855], atol=TOL)
    b = R.SceneBuilder()
    b.point_light((0, 0, 0), (1, 1, 1))
    T = lambda y: (1, 0, 0, 0, 0, 1, 0, y, 0, 0, 1, 0, 0, 0, 0, 1)  # noqa: E731
    b.plane(transform=T(-1.0), material=(0.1, 0.9, 0.9, 200.0, 1.0, 0.0, 1.0))
    b.plane(transform=T(1.0), material=(0.1, 0.9, 0.9, 200.0, 1.0, 0.0, 1.0))
    renderer.upload(b)
    c = renderer.color_at([(0, 0, 0)], [(0, 1, 0)], remaining=5)
    assert np.allclose(c[0], [11.4, 11.4, 11.4], atol=TOL)


def test_is_shadowed_known_answers(renderer, R):  # scene.rs:498-524
    renderer.upload(default_scene(R))
    L = (-10, 10, -10)
    got = renderer.is_shadowed([(0, 10, 0), (10, -10, 10), (-20, 20, -20), (-2, 2, -2)], [L] * 4)
    assert list(got) == [False, True, False, False]


def test_n1n2_and_refraction_scene(renderer, R):
    """Nested glass spheres (ray.rs:196-235 geometry) rendered through refract/reflect recursion."""
    import oracle

    M = oracle.Oracle.mat
    b, o = R.SceneBuilder(), oracle.Oracle()
    b.point_light((-10, 10, -10), (1, 1, 1))
    o.point_light((-10, 10, -10), (1, 1, 1))
    for tr, ri, refl in ((M.scale(2, 2, 2), 1.5, 0.3), (M.translate(0, 0, -0.25), 2.0, 0.0),
                         (M.translate(0, 0, 0.25), 2.5, 0.5)):
        mat = (0.1, 0.9, 0.9, 200.0, refl, 1.0, ri)
        b.sphere(transform=tr, material=mat)
        o.add("sphere", transform=tr, material=mat)
    b.plane(transform=M.translate(0, -2.5, 0), material=(0.1, 0.9, 0.9, 200.0, 0.2, 0.0, 1.0),
            pattern=b.pattern("checker", a=b.pattern("solid", color=(1, 1, 1)), b=b.pattern("solid", color=(0, 0, 0))))
    pa, pb = o.pattern("solid", color=(1, 1, 1)), o.pattern("solid", color=(0, 0, 0))
    o.add("plane", transform=M.translate(0, -2.5, 0), material=(0.1, 0.9, 0.9, 200.0, 0.2, 0.0, 1.0),
          pattern=o.pattern("checker", a=pa, b=pb))
    renderer.upload(b)
    cam_t = M.view_transform((0.3, 1.0, -6.0), (0, 0, 0), (0, 1, 0))
    W, H = 40, 30
    cam = R.camera(W, H, math.pi / 3, cam_t)
    got = renderer.render(cam, aa=1)["avg"]
    canvas, st = o.render(oracle.Oracle.camera(W, H, math.pi / 3, cam_t))
    assert st["rays"] > st["shade_events"]
    _compare(got, canvas, "nested glass")


def test_device_render_without_frame_timing(renderer, R):
    """rr_render_device into a device buffer (the bench / multi-GPU path), with and without the
    per-frame HIP event pair (RR_NO_FRAME_TIMING): the same image as rr_render, and kernel_ms is 0
    only when the events are off.  The buffer comes from the HIP runtime the library itself links
    (torch ships its own runtime, which must initialise first when both are used: bench.py)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")
    scene, _ = _yaml_pair("c2_s1024.yaml", 64, 40, 1)
    renderer.upload(scene)
    ref = renderer.render(scene.camera, aa=1)["avg"]
    nbytes = ref.size * 8
    for flags, timed in ((R._lib.RR_OUT_AVG, True), (R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING, False)):
        d = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(nbytes)) == 0
        try:
            opts = R._lib.RenderOpts(1, 5, 0, 0, 0, 1, 8, flags)
            renderer.render_device(scene.camera, opts, None, d.value, None)
            st = renderer.last_stats()  # waits for the frame
            out = np.empty_like(ref)
            assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_size_t(nbytes), 2) == 0
        finally:
            hip.hipFree(d)
        assert np.array_equal(out, ref), flags
        assert (st["kernel_ms"] > 0) == timed, st["kernel_ms"]
        assert st["rays"] == 64 * 40


NAN_CAMERA = "camera: {fov: 60, from: [0, 1, -5], to: [0, 1, -5], up: [0, 1, 0]}\n"  # from == to: NaN view


def _nan_scene(objects):
    return (NAN_CAMERA + "lights:\n  - type: point\n    color: [1, 1, 1]\n    position: [-10, 10, -10]\nscene:\n" +
            objects)


def test_nan_intersection_returns_rr_e_nan(renderer, R):
    """from == to makes view_transform's forward 0/0 (camera.rs view_transform), so every camera ray
    is NaN.  Two planes then give each ray a list of two NaN entries, which Vec::sort_by(partial_cmp()
    .unwrap()) panics on (scene.rs:104): rr_render returns RR_E_NAN (the oracle flags the same
    render), and so does one sphere (a NaN discriminant is not < 0: two NaN entries, sphere.rs:64-78).
    One plane gives one-entry lists the sort never compares: it renders without an error, as in the
    reference."""
    from oracle.scene_yaml import build_from_yaml

    for objs in ("  - type: plane\n  - type: plane\n    transforms: [{type: translate, amount: [0, -1, 0]}]\n",
                 "  - type: sphere\n"):
        text = _nan_scene(objs)
        scene = R.YamlScene(text, 16, 8, 1)
        renderer.upload(scene)
        with pytest.raises(R.RRError) as ei:
            renderer.render(scene.camera, aa=1)
        assert ei.value.code == -7, str(ei.value)  # RR_E_NAN
        st = renderer.last_stats()
        assert st["nan_rays"] == 16 * 8, st
        o, cam = build_from_yaml(text, 16, 8, 1)
        with pytest.raises(RuntimeError, match="panic"):
            o.render(cam, max_depth=5)
    for objs in ("  - type: plane\n",):
        text = _nan_scene(objs)
        scene = R.YamlScene(text, 16, 8, 1)
        renderer.upload(scene)
        got = renderer.render(scene.camera, aa=1)
        assert got["stats"]["nan_rays"] == 0
        o, cam = build_from_yaml(text, 16, 8, 1)
        canvas, _ = o.render(cam, max_depth=5)
        assert np.array_equal(got["avg"], o.aa_average(canvas, 1), equal_nan=True)


def test_area_light_png_statistically(renderer, R):
    """examples/area_light.png is one draw of the reference's thread_rng jitter (light.rs:47-65), rendered
    800x400 at aa=4 (the aa that reproduces it; aa 1-3 and 5-6 leave >30 000 jitter-free pixels
    different).  Eight jitter seeds of the GPU render: pixels whose quantised colour is the same under
    every seed do not depend on the jitter (fully lit, umbra, sky) and must equal the reference's —
    allowed: 0.1 % of them off by <= 2 levels (pixels whose rare jitter dependence eight seeds did not
    expose).  Penumbra pixels: the reference's value must lie inside the seeds' range +-2 levels for
    >= 99.5 % of them, and the mean |reference - seed mean| must stay below one level."""
    PIL = pytest.importorskip("PIL.Image")
    text = open(os.path.join(SCENES, "c5_area_light.yaml")).read()  # byte-identical to examples/area_light.yaml
    aa = 4
    scene = R.YamlScene(text, 800, 400, aa, obj_root=GOLDEN)
    renderer.upload(scene)
    Q = np.stack([R.quantize(renderer.render(scene.camera, aa=aa, seed=s)["avg"])[..., :3].astype(np.int32)
                  for s in range(8)])
    ref = np.asarray(PIL.open(os.path.join(GOLDEN, "png", "area_light.png")).convert("RGB")).astype(np.int32)
    stable = (Q == Q[0]).all(axis=0).all(axis=2)
    d = np.abs(Q[0] - ref).max(axis=2)[stable]
    pen = ~stable
    inside = ((ref >= Q.min(axis=0) - 2) & (ref <= Q.max(axis=0) + 2)).all(axis=2)[pen]
    mean_dev = float(np.abs(ref - Q.mean(axis=0))[pen].mean())
    print(f"area_light.png aa=4: {int(stable.sum())} jitter-free px, {int((d > 0).sum())} differ (max {int(d.max())}); "
          f"{int(pen.sum())} penumbra px, {float(inside.mean()):.4f} inside the seed range, mean dev {mean_dev:.3f}")
    assert stable.sum() > 300000
    assert (d > 0).sum() <= 0.001 * d.size and d.max() <= 2
    assert inside.mean() >= 0.995 and mean_dev < 1.0


def test_texture_formats_through_gpu(renderer, tmp_path):
    """Spheres textured from BMP, GIF (interlaced), TGA (run-length), PNM and interlaced PNG files (texture.rs:15-19,
    sphere uv mapping): decoded by the product front-end (png.cpp, imgfmt.cpp) on one side and by PIL in the oracle on
    the other, rendered on the GPU and in the oracle — the frames are bit-identical, with equal recursion counters."""
    from PIL import Image

    import rray_amd as R
    from oracle.scene_yaml import build_from_yaml

    rng = np.random.default_rng(23)
    ys, xs = np.mgrid[0:32, 0:64]
    base = np.stack([(xs * 4) % 256, (ys * 8) % 256, ((xs + ys) * 3) % 256], -1).astype(np.uint8)
    base ^= rng.integers(0, 32, size=base.shape, dtype=np.uint8)
    img = Image.fromarray(base, "RGB")
    img.save(tmp_path / "t.bmp")
    img.save(tmp_path / "t.gif", interlace=True)
    img.save(tmp_path / "t.tga", compression="tga_rle")
    img.save(tmp_path / "t.ppm")
    from png_helpers import png_bytes

    (tmp_path / "t.png").write_bytes(png_bytes(base, 2, 8, 1))
    files = ["t.bmp", "t.gif", "t.tga", "t.ppm", "t.png"]
    objs = "".join(
        f"  - type: sphere\n    transforms:\n      - type: scale\n        amount: [0.45, 0.45, 0.45]\n"
        f"      - type: translate\n        amount: [{-2.0 + k}, 1, 0]\n"
        f"    material:\n      pattern: {{type: image, file: '{f}'}}\n      specular: 0.3\n"
        for k, f in enumerate(files))
    text = ("camera: {fov: 60, from: [0, 1.5, -5], to: [0, 1, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [-10, 10, -10]\nscene:\n" + objs)
    W, H, aa = 96, 48, 2
    scene = R.YamlScene(text, W, H, aa, obj_root=str(tmp_path))
    o, cam = build_from_yaml(text, W, H, aa, obj_root=str(tmp_path))
    renderer.upload(scene)
    got = renderer.render(scene.camera, aa=aa, max_depth=5, canvas=True)
    canvas, st = o.render(cam, max_depth=5)
    _, exact = _compare(got["canvas"], canvas, "texture formats canvas")
    assert exact == 1.0
    assert got["stats"]["shade_events"] == st["shade_events"]

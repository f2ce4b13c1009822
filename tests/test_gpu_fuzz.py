"""Exact-cull fuzz on the GPU: seeded adversarial scenes (tests/scene_fuzz.py) rendered through the C ABI
must equal the oracle bit for bit, with the same ray / shadow-ray / shading-event counts.

The kernels test only the nodes their conservative f32 culls cannot reject; the
reference tests every primitive (scene.rs:97-106).  A margin that is too tight shows up as a missed hit —
a wrong pixel and a changed counter — in exactly the scenes the configs never render: extreme scales,
far cameras, near-parallel bundles, sheared group hierarchies, grazing planes, lights at surfaces.  A
failing seed prints its scene (tests/scene_fuzz.py builds it again from the seed alone).

The one arithmetic difference the kernels keep on purpose is the specular power: they compute the
correctly rounded x^n for integer shininess, while the reference's f64::powf is libm's
pow (<= 0.52 ulp, not always correctly rounded).  So the GPU canvas must equal, bit for bit, the oracle
with correctly rounded powers (oracle pow_mode 1, a diagnostic switch), and may differ from the
libm-pow oracle only in samples where the two oracles themselves differ (a last-ulp pow difference,
never a walk or cull error)."""
import numpy as np
import pytest

import scene_fuzz as F  # noqa: E402

pytestmark = pytest.mark.gpu
SEEDS = range(96)


@pytest.fixture(scope="module")
def renderer():
    import rray_amd

    if rray_amd.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")
    r = rray_amd.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_scene_bit_exact(renderer, seed):
    P, spec, depth, cat = F.build(seed)
    aa = 2 if seed % 3 == 0 else 1
    W, H = (24, 16) if aa == 2 else (32, 24)
    cam, ocam = F.cameras(P, spec, W * aa, H * aa)
    renderer.upload(P.b)
    got = renderer.render(cam, aa=aa, max_depth=depth, canvas=True)
    canvas, st = P.o.render(ocam, max_depth=depth)  # libm pow: the reference's own arithmetic
    P.o.set_pow_mode(1)
    canvas_cr, st_cr = P.o.render(ocam, max_depth=depth)  # correctly rounded x^n
    P.o.set_pow_mode(0)
    diff = np.argwhere((got["canvas"] != canvas_cr).any(axis=2))
    pow_only = np.argwhere((got["canvas"] != canvas).any(axis=2))
    oracles_differ = (canvas != canvas_cr).any(axis=2)
    counts = {k: (got["stats"][k], v) for k, v in (("rays", st["rays"] - st["shadow_rays"]),
                                                    ("shadow_rays", st["shadow_rays"]),
                                                    ("shade_events", st["shade_events"]))}
    ok = len(diff) == 0 and all(a == b for a, b in counts.values()) and st == st_cr
    ok = ok and all(oracles_differ[y, x] for y, x in pow_only)
    if not ok:
        print(f"seed {seed} ({cat}) {W}x{H} aa{aa}: {len(diff)} samples differ from the correctly rounded "
              f"oracle, {len(pow_only)} from the libm one; counts (gpu, oracle) {counts}")
        for y, x in diff[:10]:
            print(f"  sample ({x},{y}): gpu {got['canvas'][y, x].tolist()} oracle {canvas_cr[y, x].tolist()}")
        print("\n".join(P.log))
    elif len(pow_only):
        print(f"seed {seed} ({cat}): {len(pow_only)} samples differ from libm pow by its rounding only")
    assert ok, f"seed {seed} ({cat})"
    assert float(np.max(np.abs(got["avg"] - P.o.aa_average(canvas, aa)))) <= 1e-12


@pytest.mark.parametrize("seed", range(32))
def test_area_light_fuzz_bit_exact(renderer, seed):
    """Area lights (light.rs:47-96) with occluders at the edge of the light-hull pre-test's capsule
    (render_levels.inc area_may_shadow: events whose hull no node reaches skip their level^2 walks): the
    canvas must equal the oracle's (correctly rounded powers) bit for bit, with the same ray counts."""
    P, spec, depth, cat = F.build_area(seed)
    aa = 2 if seed % 2 else 1
    W, H = (24, 16) if aa == 2 else (40, 24)
    cam, ocam = F.cameras(P, spec, W * aa, H * aa)
    renderer.upload(P.b)
    got = renderer.render(cam, aa=aa, max_depth=depth, seed=seed, canvas=True)
    P.o.set_pow_mode(1)
    canvas_cr, st = P.o.render(ocam, max_depth=depth, seed=seed)
    P.o.set_pow_mode(0)
    diff = np.argwhere((got["canvas"] != canvas_cr).any(axis=2))
    counts = {k: (got["stats"][k], v) for k, v in (("rays", st["rays"] - st["shadow_rays"]),
                                                    ("shadow_rays", st["shadow_rays"]),
                                                    ("shade_events", st["shade_events"]))}
    ok = len(diff) == 0 and all(a == b for a, b in counts.values())
    if not ok:
        print(f"seed {seed} ({cat}) {W}x{H} aa{aa}: {len(diff)} samples differ; counts (gpu, oracle) {counts}")
        for y, x in diff[:10]:
            print(f"  sample ({x},{y}): gpu {got['canvas'][y, x].tolist()} oracle {canvas_cr[y, x].tolist()}")
        print("\n".join(P.log))
    assert ok, f"seed {seed} ({cat})"


@pytest.mark.parametrize("seed", range(48))
def test_own_skip_fuzz_bit_exact(renderer, seed):
    """The own-object skip (shadow and reflected rays skip the object they leave) at its edges
    (tests/scene_fuzz.py build_own): lights on the tangent planes of visible points, lights inside spheres, the camera
    inside a sphere, sheared spheres and scaled planes, 1e-3..1e3 spheres seen from far with narrow fields of view,
    grazing mirrors, an area light straddling tangent planes.  The canvas must equal the oracle's (correctly rounded
    powers) bit for bit, with the same ray counts."""
    P, spec, depth, cat = F.build_own(seed)
    aa = 2 if seed % 4 == 3 else 1
    W, H = (24, 16) if aa == 2 else (40, 24)
    cam, ocam = F.cameras(P, spec, W * aa, H * aa)
    renderer.upload(P.b)
    got = renderer.render(cam, aa=aa, max_depth=depth, seed=seed, canvas=True)
    P.o.set_pow_mode(1)
    canvas_cr, st = P.o.render(ocam, max_depth=depth, seed=seed)
    P.o.set_pow_mode(0)
    diff = np.argwhere((got["canvas"] != canvas_cr).any(axis=2))
    counts = {k: (got["stats"][k], v) for k, v in (("rays", st["rays"] - st["shadow_rays"]),
                                                    ("shadow_rays", st["shadow_rays"]),
                                                    ("shade_events", st["shade_events"]))}
    ok = len(diff) == 0 and all(a == b for a, b in counts.values())
    if not ok:
        print(f"seed {seed} ({cat}) {W}x{H} aa{aa}: {len(diff)} samples differ; counts (gpu, oracle) {counts}")
        for y, x in diff[:10]:
            print(f"  sample ({x},{y}): gpu {got['canvas'][y, x].tolist()} oracle {canvas_cr[y, x].tolist()}")
        print("\n".join(P.log))
    assert ok, f"seed {seed} ({cat})"

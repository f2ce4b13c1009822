"""Exact-cull fuzz on the GPU: seeded adversarial scenes (tests/scene_fuzz.py) rendered through the C ABI
must equal the oracle bit for bit, with the same ray / shadow-ray / shading-event counts.

The kernels test only the nodes their conservative f32 culls cannot reject; the
reference tests every primitive (scene.rs:97-106).  A margin that is too tight shows up as a missed hit —
a wrong pixel and a changed counter — in exactly the scenes the configs never render: extreme scales,
far cameras, near-parallel bundles, sheared group hierarchies, grazing planes, lights at surfaces.  A
failing seed prints its scene (tests/scene_fuzz.py builds it again from the seed alone)."""
import numpy as np
import pytest

import scene_fuzz as F  # noqa: E402

pytestmark = pytest.mark.gpu
SEEDS = range(48)


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
    canvas, st = P.o.render(ocam, max_depth=depth)
    diff = np.argwhere((got["canvas"] != canvas).any(axis=2))
    counts = {k: (got["stats"][k], v) for k, v in (("rays", st["rays"] - st["shadow_rays"]),
                                                    ("shadow_rays", st["shadow_rays"]),
                                                    ("shade_events", st["shade_events"]))}
    ok = len(diff) == 0 and all(a == b for a, b in counts.values())
    if not ok:
        print(f"seed {seed} ({cat}) {W}x{H} aa{aa}: {len(diff)} samples differ, counts (gpu, oracle) {counts}")
        for y, x in diff[:10]:
            print(f"  sample ({x},{y}): gpu {got['canvas'][y, x].tolist()} oracle {canvas[y, x].tolist()}")
        print("\n".join(P.log))
    assert ok, f"seed {seed} ({cat})"
    assert np.array_equal(got["avg"], P.o.aa_average(canvas, aa))

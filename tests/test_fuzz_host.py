"""Host side of the exact-cull fuzz (tests/scene_fuzz.py): every seeded adversarial scene builds the same
scene on both sides — the product's flattening (rr_scene_inspect, no device) holds the inverse the oracle
computes for every object (matrix.rs:389-412 restated twice) — and the oracle renders it to finite
values.  The GPU comparison itself is tests/test_gpu_fuzz.py."""
import ctypes as C
import os
import time

import numpy as np
import pytest

import scene_fuzz as F  # noqa: E402

SEEDS = range(96)


@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_scene_builds_identically(oracle_mod, seed):
    import rray_amd as R

    P, spec, depth, cat = F.build(seed)
    desc = P.b.desc()
    n = desc.n_objects
    inv = np.zeros((n, 16))
    node = np.zeros(n, np.int32)
    R._lib.check(R.lib().rr_scene_inspect(C.byref(desc), inv.ctypes.data_as(R._lib._D), None,
                                          node.ctypes.data_as(R._lib._I)))
    for bid, oid in P.ids.items():
        assert np.array_equal(inv[bid], np.array(P.o.inverse_of(oid))), (seed, cat, bid)
    assert (node >= 0).all()
    t = time.perf_counter()
    cam, ocam = F.cameras(P, spec, 24, 16)
    canvas, st = P.o.render(ocam, max_depth=depth, threads=min(4, os.cpu_count() or 1))
    assert np.isfinite(canvas).all(), (seed, cat)
    assert time.perf_counter() - t < 30
    print(f"seed {seed} {cat}: {n} objects, rays {st['rays']}, shade {st['shade_events']}, "
          f"lit px {float(np.mean(canvas.sum(axis=2) > 0)):.2f}")


@pytest.mark.parametrize("seed", range(32))
def test_area_fuzz_scene_builds_identically(oracle_mod, seed):
    """The area-light fuzz scenes (scene_fuzz.build_area) hold the same inverses on both sides and render to
    finite values with some light and some shadow."""
    import rray_amd as R

    P, spec, depth, cat = F.build_area(seed)
    desc = P.b.desc()
    n = desc.n_objects
    inv = np.zeros((n, 16))
    R._lib.check(R.lib().rr_scene_inspect(C.byref(desc), inv.ctypes.data_as(R._lib._D), None, None))
    for bid, oid in P.ids.items():
        assert np.array_equal(inv[bid], np.array(P.o.inverse_of(oid))), (seed, cat, bid)
    cam, ocam = F.cameras(P, spec, 24, 16)
    canvas, st = P.o.render(ocam, max_depth=depth, seed=seed)
    assert np.isfinite(canvas).all(), (seed, cat)
    assert st["shadow_rays"] > 0, (seed, cat)

"""The shadow walks' own-object skip (device_core.inc own_node, flatten.cpp mark_own_safe) against the reference's
arithmetic, on the CPU.

A lane whose hit object is a sphere or plane hit from outside skips that object's exact test in its point-light
shadow walk, when the object's transform and the hit satisfy mark_own_safe's bounds.  The claim behind it: such an
object has no entry with 0 <= t < distance on the lane's shadow ray (scene.rs:234-245 over every object), whatever the
rounding.  This test restates the rule (the same constants, on the oracle's own matrices) and asks the oracle — the
reference's algorithm op for op — for every object's entries on the shadow rays of every primary and first-bounce
hit of the fuzz scenes (tests/scene_fuzz.py: extreme scales, far cameras, tiny far objects, sheared groups, grazing
planes, lights at surfaces) and of the benchmark scenes: where the rule allows the skip, the own object must hold no
shadowing entry.  Fuzz seed 2 (a camera 1.9e4 units from 3e-3 spheres) is the case that put mark_own_safe's hit-
distance limit in: without it the reference's own hit point lies up to 2e-3 object units inside the sphere (the root's
b^2 - 4ac cancels) and the object does shadow itself.
"""
import math
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import scene_fuzz as F  # noqa: E402

EPS_F64 = 2.0 ** -52
W_OVER, EPS, SAFETY = 1e5, 1e-5, 1e3


def affine_of(o, obj):
    """The oracle's world-to-object map of obj (ancestors included) as (A_l, A_t), read back from world_to_object."""
    t = np.array(o.world_to_object(obj, (0.0, 0.0, 0.0, 1.0))[:3])
    cols = [np.array(o.world_to_object(obj, tuple(np.eye(3)[j]) + (1.0,))[:3]) - t for j in range(3)]
    return np.stack(cols, axis=1), t


def own_limit(al_mat, at):
    """mark_own_safe's largest allowed hit T = t |d|_inf, or None (flatten.cpp)."""
    al = np.abs(al_mat).sum(axis=1).max()
    atn = np.abs(at).max()
    if not (np.isfinite(al) and 0 < al <= 1e8 and np.isfinite(atn)):
        return None
    fwd = np.linalg.inv(al_mat)
    sigma_min = 1.0 / math.sqrt((fwd * fwd).sum())
    margin = EPS * sigma_min
    if not SAFETY * 4.0 * EPS_F64 * (al * (2.0 * W_OVER + 1.0) + atn) <= margin:
        return None
    tlim = (math.sqrt(margin / (12.0 * EPS_F64 * SAFETY)) - 1.01) / al
    return tlim * (1.0 - 1e-6) * 0.999 if tlim > 0 else None  # below the device's f32 rounding of the limit


def kinds_from_log(P):
    """object id -> (kind, parent) from the fuzz scene's description."""
    out = {}
    for line in P.log:
        m = re.match(r"\s*(\w+) id=(\d+) parent=(-?\d+)", line)
        if m:
            out[int(m.group(2))] = (m.group(1), int(m.group(3)))
    return out


def in_csg(kinds, obj):
    p = kinds[obj][1]
    while p >= 0:
        if kinds[p][0] == "csg":
            return True
        p = kinds[p][1]
    return False


def beyond_tangent(corners, over, n):
    """render_levels.inc area_beyond_tangent."""
    for c in corners:
        w = c - over
        size = np.abs(w).sum()
        scale = size + np.abs(over).sum() + np.abs(c).sum()
        if not (w[0] * n[0] + w[1] * n[1] + w[2] * n[2] > 1e-6 * scale and size < 1e6):
            return False
    return True


def check_scene(o, kinds, lights, rays, depth=1, areas=(), rng=None):
    """Shadow rays and reflected rays of the hits of `rays` (and of their reflections, `depth` bounces): (skips,
    violations); a reflected ray must find no entry t >= 0 on the object it leaves (reflect_own).  areas:
    (corner, u, v) of area lights, whose rays toward 16 random points of the light and its corners are checked where
    area_beyond_tangent allows the skip."""
    rng = rng or np.random.default_rng(0)
    skips = viol = 0
    limits = {}
    todo = [(r, 0) for r in rays]
    while todo:
        (org, d), lvl = todo.pop()
        xs = o.intersect(org, d)
        cand = [i for i, x in enumerate(xs) if x[0] >= 0.0]
        if not cand:
            continue
        h = min(cand, key=lambda i: (xs[i][0], i))
        c = o.prepare_computations(org, d, xs, h)
        obj = xs[h][1]
        kind, _ = kinds.get(obj, ("?", -1))
        over = np.array(c["over_point"][:3])
        n = np.array(c["normalv"][:3])
        if lvl < depth:
            todo.append(((tuple(over) + (1.0,), tuple(c["reflectv"][:3]) + (0.0,)), lvl + 1))
        if kind not in ("sphere", "plane") or in_csg(kinds, obj) or c["inside"]:
            continue
        if obj not in limits:
            limits[obj] = own_limit(*affine_of(o, obj))
        lim = limits[obj]
        T = xs[h][0] * np.abs(np.array(d[:3])).max()
        if lim is None or not T <= lim or not np.abs(over).max() <= W_OVER:
            continue
        rv = np.array(c["reflectv"][:3])
        if rv[0] * n[0] + rv[1] * n[1] + rv[2] * n[2] >= 1e-6:  # reflect_own: the reflected ray's closest-hit walk
            skips += 1
            sx = o.intersect(tuple(over) + (1.0,), tuple(rv) + (0.0,))
            if any(ob == obj and t >= 0.0 for (t, ob, _, _) in sx):
                viol += 1
        for L in lights:
            v = np.array(L) - over
            dist = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
            lv = v / dist
            ldn = lv[0] * n[0] + lv[1] * n[1] + lv[2] * n[2]
            if not (ldn >= 0.0 and dist < 1e6):
                continue
            skips += 1
            sx = o.intersect(tuple(over) + (1.0,), tuple(lv) + (0.0,))
            if any(ob == obj and 0.0 <= t < dist for (t, ob, _, _) in sx):
                viol += 1
        for corner, u, v in areas:
            corner, u, v = (np.array(a, dtype=float) for a in (corner, u, v))
            corners = [corner, corner + u, corner + v, corner + u + v]
            if not beyond_tangent(corners, over, n):
                continue
            for uf, vf in list(rng.random((16, 2))) + [(0.0, 0.0), (1.0, 0.0), (0.0, 1.0), (1.0, 1.0)]:
                tgt = corner + u * uf + v * vf
                w = tgt - over
                dist = math.sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2])
                skips += 1
                sx = o.intersect(tuple(over) + (1.0,), tuple(w / dist) + (0.0,))
                if any(ob == obj and 0.0 <= t < dist for (t, ob, _, _) in sx):
                    viol += 1
    return skips, viol


def camera_rays(ocam, W, H, step=1):
    import oracle

    return [oracle.Oracle.ray_for_pixel(ocam, px, py) for py in range(0, H, step) for px in range(0, W, step)]


@pytest.mark.parametrize("seed", range(96))
def test_own_object_never_shadows_where_skipped(seed):
    P, spec, depth, cat = F.build(seed)
    W, H = 32, 24
    _, ocam = F.cameras(P, spec, W, H)
    kinds = kinds_from_log(P)
    lights = [tuple(float(x) for x in m.groups()) for line in P.log
              for m in [re.match(r"point light \(([^,]+), ([^,]+), ([^)]+)\)", line)] if m]
    areas = [tuple(tuple(float(x) for x in g.split(",")) for g in m.groups()) for line in P.log
             for m in [re.match(r"area light corner=\(([^)]+)\) u=\(([^)]+)\) v=\(([^)]+)\)", line)] if m]
    skips, viol = check_scene(P.o, kinds, lights, camera_rays(ocam, W, H), depth=1, areas=areas)
    assert viol == 0, f"seed {seed} ({cat}): the own object shadows {viol} of {skips} skipped shadow rays"


def _fuzz_lights(P):
    lights = [tuple(float(x) for x in m.groups()) for line in P.log
              for m in [re.match(r"point light \(([^,]+), ([^,]+), ([^)]+)\)", line)] if m]
    areas = [tuple(tuple(float(x) for x in g.split(",")) for g in m.groups()) for line in P.log
             for m in [re.match(r"area light corner=\(([^)]+)\) u=\(([^)]+)\) v=\(([^)]+)\)", line)] if m]
    return lights, areas


_OWN_SKIPS = []


@pytest.mark.parametrize("seed", range(48))
def test_own_object_never_shadows_in_edge_scenes(seed):
    """tests/scene_fuzz.py build_own: the skip's edge cases (lights on tangent planes and inside spheres, the camera
    inside a sphere, sheared spheres, scaled planes, far small spheres, grazing mirrors, area lights straddling tangent
    planes), primary hits and two bounces."""
    P, spec, depth, cat = F.build_own(seed)
    _, ocam = F.cameras(P, spec, 40, 24)
    lights, areas = _fuzz_lights(P)
    skips, viol = check_scene(P.o, kinds_from_log(P), lights, camera_rays(ocam, 40, 24), depth=2, areas=areas)
    _OWN_SKIPS.append(skips)
    assert viol == 0, f"seed {seed} ({cat}): the own object shadows or blocks {viol} of {skips} skipped rays"


def test_own_edge_scenes_exercise_the_skip():
    if len(_OWN_SKIPS) < 48:
        pytest.skip("runs after the edge-scene tests (same process)")
    assert sum(_OWN_SKIPS) > 10000 and sum(1 for k in _OWN_SKIPS if k) >= 36, _OWN_SKIPS


@pytest.mark.parametrize("wl,depth", [("c2_s1024", 0), ("c3_s1024_reflect", 2)])
def test_own_skip_applies_in_the_benchmark_scenes(wl, depth):
    """The benchmark scenes (every 37th pixel of 1920 x 1080; C3's reflections to two bounces): the skip applies to
    most shadow rays, and the own object never shadows one of them.  Object ids follow creation order: the plane,
    then the 1024 spheres (scenes/make_scenes.py)."""
    from oracle import scene_yaml

    text = open(os.path.join(ROOT, "scenes", wl + ".yaml")).read()
    o, ocam = scene_yaml.build_from_yaml(text, 1920, 1080)
    kinds = {0: ("plane", -1)}
    kinds.update({k: ("sphere", -1) for k in range(1, 1025)})
    rays = camera_rays(ocam, 1920, 1080, step=37)
    skips, viol = check_scene(o, kinds, [(-10.0, 10.0, -10.0)], rays, depth=depth)
    assert viol == 0 and skips > len(rays) // 2, (skips, viol, len(rays))


def test_own_skip_area_light_scene():
    """C5's scene (scenes/c5_area_light.yaml: plane, sphere, area light; every 23rd pixel of 1920 x 1080, one bounce):
    where every corner of the light lies beyond the tangent plane the own object shadows none of the light's rays."""
    from oracle import scene_yaml

    text = open(os.path.join(ROOT, "scenes", "c5_area_light.yaml")).read()
    o, ocam = scene_yaml.build_from_yaml(text, 1920, 1080)
    kinds = {0: ("plane", -1), 1: ("sphere", -1)}
    rays = camera_rays(ocam, 1920, 1080, step=23)
    area = ((-5.0, 5.0, -5.0), (1.5, 0.0, 0.0), (0.0, 1.5, 0.0))
    skips, viol = check_scene(o, kinds, [], rays, depth=1, areas=[area])
    assert viol == 0 and skips > 0, (skips, viol)

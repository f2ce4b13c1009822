"""The area-light umbra skip (render_levels.inc area_in_umbra, flatten.cpp mark_inner_balls) against the reference's
arithmetic, on the CPU.

An event whose four light corners all lie in the cone from its over point through a sphere's inner ball, and beyond the
sphere along that cone, gets every level^2 sample shadowed without walking them.  The claim behind it: then every
sample point p of the light's parallelogram has an entry with 0 <= t < distance on that sphere (scene.rs:234-245).  This
test restates the rule — the inner ball exactly as flatten.cpp builds it (centre and radius rounded to f32 as stored),
the kernel's conditions with their margins, and the sphere's true outer radius in place of the device's inflated cull
radius (which only makes the device claim less) — and asks the oracle, the reference's algorithm op for op, whether the
segments to the corners, the centre and 40 random points of the parallelogram are shadowed wherever the rule claims
the umbra: on C5's scene (points on the floor around the sphere's shadow, and on the sphere) and on 200 random scenes of
one sheared, rotated ellipsoid under a random area light.  None may be unshadowed, and the rule must claim a share of
the points that walk (else the skip would do nothing).
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def affine_of(o, obj):
    t = np.array(o.world_to_object(obj, (0.0, 0.0, 0.0, 1.0))[:3])
    cols = [np.array(o.world_to_object(obj, tuple(np.eye(3)[j]) + (1.0,))[:3]) - t for j in range(3)]
    return np.stack(cols, axis=1), t


def inner_ball(al, at):
    """flatten.cpp mark_inner_balls: (centre as f32, radius as f32 rounded down), or None."""
    c = -np.linalg.solve(al, at)
    smax = np.linalg.svd(al, compute_uv=False)[0]
    res = float(np.linalg.norm(al @ c + at))
    if not (np.all(np.isfinite(c)) and smax > 0 and res < 0.5):
        return None
    cf = c.astype(np.float32)
    shift = float(np.linalg.norm(cf.astype(np.float64) - c))
    scale = float(np.abs(c).sum())
    r = ((1.0 - res) / smax) * (1.0 - 1e-6) - 2.0 * shift - 1e-9 * (scale + 1.0 / smax)
    if not r > 0:
        return None
    return cf.astype(np.float64), float(np.nextafter(np.float32(r), np.float32(0.0)))


def umbra(o, ball, r_out, corners):
    """render_levels.inc area_in_umbra for one node (the kernel's expressions and margins)."""
    c, r = ball
    w = c - o
    L = math.sqrt(float(w @ w))
    if not (L > r * (1.0 + 1e-6) and L < 1e3 * r):
        return False
    for q in corners:
        v = q - o
        x = np.cross(v, w)
        if not (float(x @ x) < (r * r) * float(v @ v) * (1.0 - 1e-6) and float(v @ w) > L * (L + r_out) * (1.0 + 1e-6)):
            return False
    return True


def check(o, sphere_id, corner, u, v, points, rng, n_samples=40):
    al, at = affine_of(o, sphere_id)
    ball = inner_ball(al, at)
    assert ball is not None
    r_out = float(np.linalg.svd(np.linalg.inv(al), compute_uv=False)[0])  # the sphere's true outer radius
    corner, u, v = np.array(corner, float), np.array(u, float), np.array(v, float)
    corners = [corner, corner + u, corner + v, corner + u + v]
    claims = violations = 0
    for p in points:
        if not umbra(np.array(p, float), ball, r_out, corners):
            continue
        claims += 1
        samples = corners + [corner + 0.5 * u + 0.5 * v] + [corner + a * u + b * v for a, b in rng.random((n_samples, 2))]
        violations += sum(not o.is_shadowed(tuple(p) + (1.0,), tuple(s) + (1.0,)) for s in samples)
    return claims, violations


def test_umbra_rule_on_c5_scene():
    from oracle import scene_yaml

    text = open(os.path.join(ROOT, "scenes", "c5_area_light.yaml")).read()
    o, _ = scene_yaml.build_from_yaml(text, 64, 36)
    rng = np.random.default_rng(1)
    # the floor (y = 0, over points EPS above) around the sphere's shadow, and points on the sphere's lower half
    pts = [(x, 1e-5, z) for x in np.linspace(-1.5, 3.5, 41) for z in np.linspace(-1.5, 3.5, 41)]
    for th in np.linspace(0.1, 3.0, 15):
        for ph in np.linspace(0.0, 2 * math.pi, 24, endpoint=False):
            n = np.array([math.sin(th) * math.cos(ph), -math.cos(th), math.sin(th) * math.sin(ph)])
            pts.append(tuple(np.array([0.0, 1.0, 0.0]) + n * (1.0 + 1e-5)))
    claims, viol = check(o, 1, (-5.0, 5.0, -5.0), (1.5, 0.0, 0.0), (0.0, 1.5, 0.0), pts, rng)
    assert viol == 0 and claims > 100, (claims, viol)


def test_umbra_rule_fuzz():
    from oracle.oracle import Oracle

    rng = np.random.default_rng(7)
    M = Oracle.mat
    total_claims = 0
    for k in range(200):
        o = Oracle()
        s = rng.uniform(0.05, 3.0, 3) if k % 2 else np.full(3, rng.uniform(0.05, 3.0))
        t = M.translate(*rng.uniform(-2, 2, 3))
        r = M.rotate(rng.integers(0, 3), rng.uniform(0, 2 * math.pi))
        sh = M.shear(*(rng.uniform(-0.5, 0.5, 6) if k % 3 == 0 else np.zeros(6)))
        tr = M.multiply(t, M.multiply(r, M.multiply(sh, M.scale(*s))))
        sid = o.add("sphere", transform=tr)
        centre = np.array(M.multiply_tuple(tr, (0.0, 0.0, 0.0, 1.0))[:3])
        size = float(np.max(s)) * (1.5 if k % 3 == 0 else 1.0)
        # the light somewhere above, the points on the opposite side: many segments cross the ellipsoid
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        dist = rng.uniform(3.0, 30.0) * size
        lw = rng.uniform(0.05, 1.5) * size
        u = np.cross(d, [0.3, 1.0, 0.2])
        u = u / np.linalg.norm(u) * lw
        v = np.cross(d, u)
        v = v / np.linalg.norm(v) * lw * rng.uniform(0.3, 1.0)
        corner = centre + d * dist - 0.5 * u - 0.5 * v
        o.area_light(tuple(corner), tuple(u), tuple(v), (1.0, 1.0, 1.0), 3)
        pts = [tuple(centre - d * rng.uniform(1.0, 6.0) * size + rng.normal(size=3) * size * rng.uniform(0.05, 1.5))
               for _ in range(60)]
        claims, viol = check(o, sid, corner, u, v, pts, rng, n_samples=20)
        assert viol == 0, (k, claims, viol)
        total_claims += claims
    assert total_claims > 500, total_claims

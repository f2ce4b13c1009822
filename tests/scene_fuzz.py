"""Seeded adversarial scenes for the exact-cull fuzz (tests/test_gpu_fuzz.py, tests/test_fuzz_host.py).

Every scene is built twice from the same numbers: through the product's SceneBuilder (C ABI descriptor)
and through the oracle (the CPU restatement of the reference, test infrastructure).  The kernels cull
nodes with conservative f32 tests (bundle cones, lane line tests, the far-origin shift, inflated cull
spheres; DESIGN.md §3.5, device_core.inc, flatten.cpp make_cull) whose slacks are hand-derived; the
reference tests every primitive for every ray (scene.rs:97-106).  These scenes go where the benchmark
configs never do:

  scales    spheres from 1e-3 to 1e4 units, huge ones far away, a floor
  far_cam   the camera 1e3-1e5 units outside the scene's bounding sphere, narrow field of view (the
            far-origin shift of the bundles, device_core.inc make_bundle)
  tiny_far  objects of 1e-3 units 1e3-1e5 away, the camera aimed at them with a tiny field of view
            (near-parallel bundles, cull radii at the edge of f32 resolution)
  groups    nested groups with non-uniform scale and shear holding spheres, triangles and smooth
            triangles (ancestor chains, group AABBs, transformed cull spheres)
  grazing   planes tilted a few milli-radians off the view direction, camera just above a floor
  lights    lights inside / next to surfaces, reflective everywhere, glass (the n1/n2 walk's two-sided
            culls), recursion depth 5
  many      600-900 spheres of mixed scale (culls too large for LDS: the global-memory cull kernels)
  general   cubes and cylinders inside sheared groups (the G = 2 kernels)

Shininess is 200 everywhere so the specular power takes the correctly rounded path:
any difference from the oracle is then a walk / cull error, never a last-ulp `pow`.
"""
import math

import numpy as np

CATEGORIES = ["scales", "far_cam", "tiny_far", "groups", "grazing", "lights", "many", "general"]
SHININESS = 200.0


class Pair:
    """One scene on both sides: product SceneBuilder + oracle.Oracle, identical inputs."""

    def __init__(self):
        import oracle
        import rray_amd as R

        self.b = R.SceneBuilder()
        self.o = oracle.Oracle()
        self.M = oracle.Oracle.mat
        self.ids = {}  # builder id -> oracle id
        self.log = []  # printable description (failing seeds print it)

    def _mat(self, m7, color):
        pb = self.b.pattern("solid", color=color)
        po = self.o.pattern("solid", color=color)
        return pb, po

    def obj(self, kind, tr, m7=None, color=(0.8, 0.5, 0.3), parent=-1):
        po_parent = self.ids[parent] if parent >= 0 else -1
        if kind == "group":
            bid = self.b.group(transform=tr, parent=parent)
            oid = self.o.add("group", po_parent, tr)
        else:
            pb, po = self._mat(m7, color)
            if kind == "sphere":
                bid = self.b.sphere(transform=tr, material=m7, pattern=pb, parent=parent)
            elif kind == "plane":
                bid = self.b.plane(transform=tr, material=m7, pattern=pb, parent=parent)
            elif kind == "cube":
                bid = self.b.cube(transform=tr, material=m7, pattern=pb, parent=parent)
            else:
                raise ValueError(kind)
            oid = self.o.add(kind, po_parent, tr, m7, po)
        self.ids[bid] = oid
        self.log.append(f"{kind} id={bid} parent={parent} tr={np.round(tr, 6).tolist()} mat={m7}")
        return bid

    def cylinder(self, tr, m7, color, minimum, maximum, closed, parent=-1):
        pb, po = self._mat(m7, color)
        bid = self.b.cylinder(minimum, maximum, closed, transform=tr, material=m7, pattern=pb, parent=parent)
        oid = self.o.add("cylinder", self.ids[parent] if parent >= 0 else -1, tr, m7, po)
        self.o.set_shape_params(oid, minimum, maximum, closed)
        self.ids[bid] = oid
        self.log.append(f"cylinder id={bid} parent={parent} [{minimum},{maximum}] closed={closed} "
                        f"tr={np.round(tr, 6).tolist()} mat={m7}")
        return bid

    def triangle(self, p1, p2, p3, m7, color, parent=-1, normals=None):
        pb, po = self._mat(m7, color)
        op = self.ids[parent] if parent >= 0 else -1
        if normals is None:
            bid = self.b.triangle(p1, p2, p3, material=m7, pattern=pb, parent=parent)
            oid = self.o.add_triangle(p1, p2, p3, op)
        else:
            bid = self.b.smooth_triangle(p1, p2, p3, *normals, material=m7, pattern=pb, parent=parent)
            oid = self.o.add_smooth_triangle(p1, p2, p3, *normals, parent=op)
        self.o.set_material(oid, m7, po)
        self.ids[bid] = oid
        self.log.append(f"{'smooth_' if normals else ''}triangle id={bid} parent={parent} "
                        f"p={np.round([p1, p2, p3], 6).tolist()} mat={m7}")
        return bid

    def light(self, pos, color=(1.0, 1.0, 1.0)):
        pos = tuple(float(x) for x in pos)
        self.b.point_light(pos, color)
        self.o.point_light(pos, color)
        self.log.append(f"point light {pos}")

    def area_light(self, corner, u, v, level, color=(1.0, 1.0, 1.0)):
        corner, u, v = (tuple(float(x) for x in a) for a in (corner, u, v))
        self.b.area_light(corner, u, v, color, int(level))
        self.o.area_light(corner, u, v, color, int(level))
        self.log.append(f"area light corner={corner} u={u} v={v} level={level}")


def _mul(M, *ts):
    """ts applied first to last (the YAML transform list order, scene_builder_yaml.rs:218-224)."""
    m = M.identity()
    for t in ts:
        m = M.multiply(t, m)
    return m


def _material(rng, reflective_p=0.3, glass_p=0.0):
    refl = float(rng.choice([0.0, 0.3, 0.5, 0.9])) if rng.random() < reflective_p else 0.0
    transp, ri = (0.0, 1.0)
    if rng.random() < glass_p:
        transp, ri = float(rng.choice([0.5, 0.9, 1.0])), float(rng.choice([1.33, 1.5, 2.4]))
    return (float(rng.uniform(0.05, 0.3)), float(rng.uniform(0.3, 0.9)), float(rng.uniform(0.0, 0.9)), SHININESS,
            refl, transp, ri)


def _color(rng):
    return tuple(float(round(x, 3)) for x in rng.uniform(0.05, 1.0, 3))


def _rot(M, rng):
    return _mul(M, M.rotate("x", float(rng.uniform(-math.pi, math.pi))), M.rotate("y", float(rng.uniform(-math.pi, math.pi))),
                M.rotate("z", float(rng.uniform(-math.pi, math.pi))))


def _logu(rng, lo, hi):
    return float(math.exp(rng.uniform(math.log(lo), math.log(hi))))


def _unit(rng):
    v = rng.standard_normal(3)
    return v / np.linalg.norm(v)


def build(seed):
    """-> (Pair, camera spec dict(from_, to, up, fov), max_depth, category)."""
    rng = np.random.default_rng(10_000 + seed)
    cat = CATEGORIES[seed % len(CATEGORIES)]
    P = Pair()
    M = P.M
    depth = 5
    frm, to, fov = (0.0, 3.0, -30.0), (0.0, 0.0, 0.0), 1.0

    def sphere_at(c, s, m7=None, parent=-1, aniso=False):
        sc = (s * rng.uniform(0.2, 5.0), s, s * rng.uniform(0.2, 5.0)) if aniso else (s, s, s)
        tr = _mul(M, M.scale(*sc), _rot(M, rng), M.translate(*[float(x) for x in c])) if aniso else \
            _mul(M, M.scale(*sc), M.translate(*[float(x) for x in c]))
        return P.obj("sphere", tr, m7 or _material(rng), _color(rng), parent)

    if cat == "scales":
        P.obj("plane", M.translate(0.0, -2.0, 0.0), _material(rng), _color(rng))
        for _ in range(int(rng.integers(40, 160))):
            s = _logu(rng, 1e-3, 10.0)
            sphere_at(rng.uniform(-15, 15, 3) * [1, 0.3, 1] + [0, 2, 0], s, aniso=rng.random() < 0.3)
        for _ in range(int(rng.integers(2, 6))):  # huge and far: 1e2-1e4 units at 1e3-1e5
            d = _logu(rng, 1e3, 1e5)
            s = min(_logu(rng, 1e2, 1e4), 0.5 * d)
            dirv = _unit(rng) * [1, 0.3, 1] + [0, 0.1, 1.0]
            sphere_at(dirv / np.linalg.norm(dirv) * d, s)
        P.light(rng.uniform(-20, 20, 3) + [0, 25, -10])
        frm, fov = (float(rng.uniform(-5, 5)), float(rng.uniform(1, 8)), -30.0), float(rng.uniform(0.6, 1.3))
    elif cat == "far_cam":
        for _ in range(int(rng.integers(30, 120))):
            sphere_at(rng.uniform(-5, 5, 3), _logu(rng, 0.05, 2.0), aniso=rng.random() < 0.2)
        if rng.random() < 0.5:
            P.obj("plane", M.translate(0.0, -5.5, 0.0), _material(rng), _color(rng))
        d = _logu(rng, 1e3, 1e5)
        v = _unit(rng) * d
        frm, to = tuple(float(x) for x in v), tuple(float(x) for x in rng.uniform(-1, 1, 3))
        fov = float(2.0 * math.atan(9.0 / d))
        P.light(rng.uniform(-30, 30, 3) + [0, 40, 0])
        if rng.random() < 0.5:
            P.light(np.array(frm) * 0.5 + rng.uniform(-3, 3, 3))
    elif cat == "tiny_far":
        d = _logu(rng, 1e3, 1e5)
        s = _logu(rng, 1e-3, 1e-2)
        dirv = _unit(rng)
        target = dirv * d
        for _ in range(int(rng.integers(20, 60))):
            sphere_at(target + rng.uniform(-8, 8, 3) * s, s * rng.uniform(0.3, 2.0), aniso=rng.random() < 0.3)
        for _ in range(int(rng.integers(0, 6))):  # triangles of the same scale next to them
            c = target + rng.uniform(-6, 6, 3) * s
            P.triangle(*(tuple(float(x) for x in c + rng.uniform(-2, 2, 3) * s) for _ in range(3)), _material(rng),
                       _color(rng))
        frm, to = (0.0, 0.0, 0.0), tuple(float(x) for x in target)
        fov = float(2.0 * math.atan(12.0 * s / d))
        P.light(target + _unit(rng) * s * 30)
        P.light(_unit(rng) * d * 2)
    elif cat == "groups":
        P.obj("plane", M.translate(0.0, -3.0, 0.0), _material(rng), _color(rng))

        def fill(parent, level):
            for _ in range(int(rng.integers(2, 5))):
                r = rng.random()
                if level < 3 and r < 0.35:
                    tr = _mul(M, M.scale(*rng.uniform(0.1, 4.0, 3)),
                              M.shear(*[float(x) for x in rng.uniform(-1.5, 1.5, 6) * (rng.random() < 0.6)]),
                              _rot(M, rng), M.translate(*[float(x) for x in rng.uniform(-3, 3, 3)]))
                    g = P.obj("group", tr, parent=parent)
                    fill(g, level + 1)
                elif r < 0.7:
                    sphere_at(rng.uniform(-2, 2, 3), _logu(rng, 0.01, 1.0), parent=parent, aniso=rng.random() < 0.5)
                else:
                    c = rng.uniform(-2, 2, 3)
                    s = _logu(rng, 0.01, 1.5)
                    pts = [tuple(float(x) for x in c + rng.uniform(-1, 1, 3) * s) for _ in range(3)]
                    nrm = None
                    if rng.random() < 0.5:
                        nrm = [tuple(float(x) for x in _unit(rng)) for _ in range(3)]
                    for _ in range(int(rng.integers(1, 4))):
                        P.triangle(*pts, _material(rng), _color(rng), parent=parent, normals=nrm)
                        pts = [pts[1], pts[2], tuple(float(x) for x in c + rng.uniform(-1, 1, 3) * s)]

        for _ in range(int(rng.integers(2, 5))):
            tr = _mul(M, M.scale(*rng.uniform(0.2, 3.0, 3)), M.shear(*[float(x) for x in rng.uniform(-1, 1, 6)]),
                      _rot(M, rng), M.translate(*[float(x) for x in rng.uniform(-6, 6, 3)]))
            fill(P.obj("group", tr), 1)
        P.light(rng.uniform(-20, 20, 3) + [0, 25, -10])
        frm, fov = (float(rng.uniform(-6, 6)), float(rng.uniform(2, 10)), -25.0), float(rng.uniform(0.6, 1.2))
    elif cat == "grazing":
        h = _logu(rng, 1e-3, 0.5)
        for _ in range(int(rng.integers(1, 4))):
            tilt = float(rng.uniform(-5e-3, 5e-3))
            tr = _mul(M, M.rotate("x", tilt), M.rotate("z", float(rng.uniform(-5e-3, 5e-3))),
                      M.translate(0.0, float(rng.uniform(-0.05, 0.05)), 0.0))
            P.obj("plane", tr, _material(rng, reflective_p=0.6), _color(rng))
        for _ in range(int(rng.integers(10, 60))):
            s = _logu(rng, 0.01, 2.0)
            sphere_at((rng.uniform(-30, 30), s * rng.uniform(-0.5, 1.5), rng.uniform(1, 400)), s)
        frm, to = (0.0, h, -5.0), (float(rng.uniform(-1, 1)), h * float(rng.uniform(0.0, 1.0)), 200.0)
        fov = float(rng.uniform(0.2, 1.0))
        P.light((float(rng.uniform(-30, 30)), float(_logu(rng, 0.01, 30.0)), float(rng.uniform(-10, 100))))
    elif cat == "lights":
        P.obj("plane", M.identity(), _material(rng, reflective_p=0.8), _color(rng))
        centers = []
        for _ in range(int(rng.integers(6, 25))):
            s = _logu(rng, 0.1, 2.0)
            c = np.array([rng.uniform(-6, 6), s, rng.uniform(-2, 10)])
            centers.append((c, s))
            sphere_at(c, s, m7=_material(rng, reflective_p=0.8, glass_p=0.3))
        for _ in range(int(rng.integers(1, 3))):  # inside a sphere, or just off its surface
            c, s = centers[int(rng.integers(len(centers)))]
            off = s * (rng.uniform(0.0, 0.8) if rng.random() < 0.4 else 1.0 + _logu(rng, 1e-6, 1e-2))
            P.light(c + _unit(rng) * off)
        if rng.random() < 0.5:
            P.light((float(rng.uniform(-5, 5)), float(_logu(rng, 1e-5, 1e-2)), float(rng.uniform(0, 8))))  # near the floor
        frm, fov = (float(rng.uniform(-4, 4)), float(rng.uniform(1, 6)), -12.0), float(rng.uniform(0.7, 1.3))
    elif cat == "many":
        P.obj("plane", M.translate(0.0, -1.0, 0.0), _material(rng), _color(rng))
        for _ in range(int(rng.integers(600, 900))):
            sphere_at(rng.uniform(-20, 20, 3) * [1, 0.4, 1] + [0, 3, 10], _logu(rng, 5e-3, 1.5))
        P.light(rng.uniform(-20, 20, 3) + [0, 30, -10])
        frm, fov = (float(rng.uniform(-5, 5)), float(rng.uniform(2, 12)), -20.0), float(rng.uniform(0.7, 1.3))
        to = (0.0, 2.0, 10.0)
    elif cat == "general":
        P.obj("plane", M.translate(0.0, -2.0, 0.0), _material(rng), _color(rng))
        for _ in range(int(rng.integers(2, 5))):
            tr = _mul(M, M.scale(*rng.uniform(0.3, 3.0, 3)), M.shear(*[float(x) for x in rng.uniform(-1, 1, 6)]),
                      _rot(M, rng), M.translate(*[float(x) for x in rng.uniform(-5, 5, 3)]))
            g = P.obj("group", tr)
            for _ in range(int(rng.integers(2, 6))):
                s = _logu(rng, 0.02, 1.0)
                t = _mul(M, M.scale(*(s * rng.uniform(0.3, 3.0, 3))), _rot(M, rng),
                         M.translate(*[float(x) for x in rng.uniform(-2, 2, 3)]))
                if rng.random() < 0.5:
                    P.obj("cube", t, _material(rng), _color(rng), parent=g)
                else:
                    lo = float(rng.uniform(-2, 0))
                    P.cylinder(t, _material(rng), _color(rng), lo, lo + float(rng.uniform(0.1, 3)), bool(rng.random() < 0.5),
                               parent=g)
            for _ in range(int(rng.integers(0, 4))):
                sphere_at(rng.uniform(-2, 2, 3), _logu(rng, 0.01, 1.0), parent=g)
        P.light(rng.uniform(-20, 20, 3) + [0, 25, -10])
        frm, fov = (float(rng.uniform(-6, 6)), float(rng.uniform(2, 10)), -25.0), float(rng.uniform(0.6, 1.2))
    up = (0.0, 1.0, 0.0)
    fwd = np.array(to) - np.array(frm)
    if abs(fwd[1]) > 0.99 * np.linalg.norm(fwd):
        up = (1.0, 0.0, 0.0)
    P.log.append(f"camera from={frm} to={to} up={up} fov={fov} depth={depth}")
    return P, {"from_": tuple(float(x) for x in frm), "to": tuple(float(x) for x in to), "up": up, "fov": fov}, depth, cat


def build_area(seed):
    """Area-light scenes for the light-hull pre-test (render_levels.inc area_may_shadow): occluders placed just
    inside and just outside the capsule around the segment from a floor point to the light's centre, tilted and
    light-side planes, skewed / tiny / huge light parallelograms, groups and cubes.  -> (Pair, camera spec, depth,
    category)."""
    rng = np.random.default_rng(20_000 + seed)
    P = Pair()
    M = P.M
    kind = seed % 4
    # the light: a parallelogram above the scene (sometimes skewed, tiny or huge), a few cells per side
    size = [0.3, 1.5, 6.0, 1e-3][int(rng.integers(4))]
    corner = np.array([rng.uniform(-6, 6), rng.uniform(4, 9), rng.uniform(-8, 2)])
    u = np.array([1.0, 0.0, 0.0]) * size
    v = (np.array([0.0, 1.0, 0.0]) if rng.random() < 0.5 else _unit(rng)) * size * rng.uniform(0.3, 1.5)
    if rng.random() < 0.4:
        u = _unit(rng) * size
    level = int(rng.integers(1, 5))
    P.area_light(corner, u, v, level)
    qc = corner + 0.5 * u + 0.5 * v
    qr = 0.5 * max(np.linalg.norm(u + v), np.linalg.norm(u - v))
    # the floor, tilted at times; a second plane near the light's side at times
    tilt = float(rng.uniform(-0.3, 0.3)) if rng.random() < 0.4 else 0.0
    P.obj("plane", _mul(M, M.rotate("z", tilt)), _material(rng, reflective_p=0.5), _color(rng))
    if kind == 1:  # a wall the light's hull straddles or just misses
        P.obj("plane", _mul(M, M.rotate("x", math.pi / 2), M.translate(0.0, 0.0, float(corner[2] + rng.uniform(-0.5, 0.5)))),
              _material(rng), _color(rng))
    parent = -1
    if kind == 2:
        parent = P.obj("group", _mul(M, M.scale(*rng.uniform(0.5, 2.0, 3)), M.translate(*rng.uniform(-1, 1, 3))))
    for _ in range(int(rng.integers(2, 9))):
        # a floor point in view, the segment to the light centre, an occluder at distance ~ r + qr from it
        fp = np.array([rng.uniform(-3, 3), 0.0, rng.uniform(-1, 5)])
        t = rng.uniform(0.1, 0.9)
        a = fp + t * (qc - fp)
        r = _logu(rng, 0.05, 1.0)
        off = (r + qr * t) * (1.0 + float(rng.choice([-1e-3, 1e-6, 1e-3, 0.05, -0.05])))
        c = a + _unit(rng) * off
        if kind == 3 and rng.random() < 0.5:
            tr = _mul(M, M.scale(r, r, r), _rot(M, rng), M.translate(*[float(x) for x in c]))
            P.obj("cube", tr, _material(rng, reflective_p=0.5), _color(rng), parent=parent)
        else:
            P.obj("sphere", _mul(M, M.scale(r, r, r), M.translate(*[float(x) for x in c])),
                  _material(rng, reflective_p=0.5), _color(rng), parent)
    if rng.random() < 0.3:
        P.light(qc + rng.uniform(-2, 2, 3))
    frm = (float(rng.uniform(-2, 2)), float(rng.uniform(1.5, 4)), -6.0)
    to = (0.0, 0.5, 2.0)
    fov = float(rng.uniform(0.8, 1.2))
    P.log.append(f"camera from={frm} to={to} fov={fov} depth=3")
    return P, {"from_": frm, "to": to, "up": (0.0, 1.0, 0.0), "fov": fov}, 3, f"area{kind}"


def build_own(seed):
    """Scenes for the own-object skip (shadow and reflected rays skip the object they leave): lights on
    or next to the tangent planes of the spheres the camera sees (light . normal ~ 0), lights inside spheres, the camera
    inside a sphere (inside hits: no skip), anisotropic and sheared spheres, tilted and scaled planes, spheres from 1e-3
    to 1e3 units, far cameras with narrow fields of view (the hit-distance limit of flatten.cpp mark_own_safe), mirrors
    viewed at grazing angles, an area light straddling a sphere's tangent planes.  -> (Pair, camera spec, depth,
    category)."""
    rng = np.random.default_rng(30_000 + seed)
    P = Pair()
    M = P.M
    kind = seed % 6
    cat = ["tangent_light", "light_inside", "camera_inside", "aniso_planes", "far_small", "area_straddle"][kind]
    depth = 4
    frm, to, fov = (0.0, 2.0, -8.0), (0.0, 0.5, 0.0), 1.0
    centres = []
    for _ in range(int(rng.integers(3, 9))):
        r = _logu(rng, 0.2, 1.5)
        c = np.array([rng.uniform(-3, 3), r * rng.uniform(0.5, 1.5), rng.uniform(-2, 3)])
        if kind == 3 and rng.random() < 0.6:
            tr = _mul(M, M.scale(r * rng.uniform(0.2, 3.0), r, r * rng.uniform(0.2, 3.0)), _rot(M, rng),
                      M.shear(*[float(x) for x in rng.uniform(-0.5, 0.5, 6)]), M.translate(*[float(x) for x in c]))
        else:
            tr = _mul(M, M.scale(r, r, r), M.translate(*[float(x) for x in c]))
        P.obj("sphere", tr, _material(rng, reflective_p=0.6), _color(rng))
        centres.append((c, r))
    tilt = float(rng.uniform(-0.2, 0.2)) if kind == 3 else 0.0
    sc = float(rng.choice([1.0, 1e-3, 50.0])) if kind == 3 else 1.0
    P.obj("plane", _mul(M, M.scale(sc, sc, sc), M.rotate("z", tilt)), _material(rng, reflective_p=0.6), _color(rng))
    c, r = centres[0]
    if kind == 0:  # lights on the tangent planes of points the camera sees: light . normal ~ 0 at those points
        for _ in range(2):
            n = _unit(rng)
            n[2] = -abs(n[2])  # facing the camera
            n /= np.linalg.norm(n)
            t = np.cross(n, _unit(rng))
            t /= np.linalg.norm(t)
            P.light(c + r * n + t * rng.uniform(2, 10) + n * float(rng.choice([0.0, 1e-9, -1e-9, 1e-6])))
    elif kind == 1:  # a light inside a sphere, another just above a surface
        P.light(c + _unit(rng) * r * 0.5)
        n = _unit(rng)
        P.light(c + n * r * (1.0 + 1e-7))
    elif kind == 2:  # the camera inside a big sphere (glass-free: inside hits shade the inner wall)
        P.obj("sphere", _mul(M, M.scale(30.0, 30.0, 30.0)), _material(rng, reflective_p=0.6), _color(rng))
        P.light(rng.uniform(-5, 5, 3) + [0, 8, 0])
    elif kind == 3:
        P.light(rng.uniform(-10, 10, 3) + [0, 12, -6])
    elif kind == 4:  # spheres from 1e-3 to 1e3 units, seen from 10^2..10^4.5 units away with a narrow field of view
        s = _logu(rng, 1e-3, 1e3)
        for _ in range(4):
            P.obj("sphere", _mul(M, M.scale(s, s, s), M.translate(*[float(x) for x in rng.uniform(-3, 3, 3) * s])),
                  _material(rng, reflective_p=0.6), _color(rng))
        P.light(rng.uniform(-10, 10, 3) * s + [0, 12 * s, 0])
        dist = _logu(rng, 1e2, 3e4) * max(s, 1.0)
        frm = tuple(float(x) for x in _unit(rng) * dist)
        to = (0.0, 0.0, 0.0)
        fov = float(8.0 * s / dist)
    else:  # an area light whose parallelogram straddles the tangent planes of the first sphere's visible points
        n = np.array([0.0, 0.3, -1.0])
        n /= np.linalg.norm(n)
        q = c + r * n
        u = np.cross(n, [0.0, 1.0, 0.0])
        u /= np.linalg.norm(u)
        P.area_light(q + n * float(rng.uniform(-0.5, 0.5)) - u * 2.0 + np.array([0.0, 1.5, 0.0]), u * 4.0,
                     np.array([0.0, 1.0, 0.0]) * float(rng.uniform(0.5, 2.0)), int(rng.integers(2, 5)))
        depth = 3
    if kind in (0, 1, 3) and rng.random() < 0.5:  # grazing view of a mirror: the camera near a sphere's silhouette
        frm = tuple(float(x) for x in c + np.array([r * 1.02, 0.0, -6.0]))
        to = tuple(float(x) for x in c + np.array([r, 0.0, 0.0]))
        fov = 0.3
    if kind == 2:
        frm, to, fov = (0.0, 1.0, -5.0), (0.0, 0.5, 2.0), 1.2
    P.log.append(f"camera from={frm} to={to} fov={fov} depth={depth}")
    return P, {"from_": tuple(float(x) for x in frm), "to": tuple(float(x) for x in to), "up": (0.0, 1.0, 0.0),
               "fov": float(fov)}, depth, cat


def cameras(P, spec, W, H):
    """Product and oracle cameras from the same view_transform (the oracle's matrix.rs restatement)."""
    import oracle
    import rray_amd as R

    t = P.M.view_transform(spec["from_"], spec["to"], spec["up"])
    return R.camera(W, H, spec["fov"], t), oracle.Oracle.camera(W, H, spec["fov"], t)

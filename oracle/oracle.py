"""ctypes binding of liboracle (rray_oracle.cpp) — TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path():
    return os.path.join(HERE, "_build", "librray_oracle.so")


def build_oracle(force=False):
    """Compile the oracle with its Makefile (g++, -ffp-contract=off)."""
    if force or not os.path.exists(lib_path()) or (
        os.path.getmtime(lib_path()) < os.path.getmtime(os.path.join(HERE, "rray_oracle.cpp"))
    ):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return lib_path()


_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int)


class OrcStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "rays", "shadow_rays", "sphere_tests", "plane_tests", "tri_tests", "group_tests",
        "group_hits", "cube_tests", "cyl_tests", "cone_tests", "csg_tests", "shade_events", "nan_sorts",
        "torus_tests")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class OracleCamera(C.Structure):
    _fields_ = [("hsize", C.c_int64), ("vsize", C.c_int64), ("field_of_view", C.c_double),
                ("pixel_size", C.c_double), ("half_width", C.c_double), ("half_height", C.c_double),
                ("transform", C.c_double * 16)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        build_oracle()
        L = C.CDLL(lib_path())
        L.orc_world_new.restype = C.c_void_p
        L.orc_world_free.argtypes = [C.c_void_p]
        for n in ("orc_add_object",):
            getattr(L, n).argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_add_triangle.argtypes = [C.c_void_p, C.c_int, _D, _D, _D]
        L.orc_add_smooth_triangle.argtypes = [C.c_void_p, C.c_int, _D, _D, _D, _D, _D, _D]
        L.orc_load_obj.argtypes = [C.c_void_p, C.c_char_p, C.c_int, _D, C.c_int]
        L.orc_set_transform.argtypes = [C.c_void_p, C.c_int, _D]
        L.orc_set_material.argtypes = [C.c_void_p, C.c_int, _D, C.c_int]
        L.orc_pattern_new.argtypes = [C.c_void_p, C.c_int, _D, C.c_int, C.c_int, C.c_double, _D]
        L.orc_add_point_light.argtypes = [C.c_void_p, _D, _D]
        L.orc_add_area_light.argtypes = [C.c_void_p, _D, _D, _D, _D, C.c_int]
        L.orc_remove_light.argtypes = [C.c_void_p, C.c_int]
        L.orc_num_children.argtypes = [C.c_void_p, C.c_int]
        L.orc_num_objects.argtypes = [C.c_void_p]
        L.orc_num_patterns.argtypes = [C.c_void_p]
        L.orc_add_texture.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint8)]
        L.orc_texture_color.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.POINTER(C.c_uint8)]
        L.orc_uv_mapping.argtypes = [C.c_void_p, C.c_int, _D, _D]
        for n, k in (("quartic", 5), ("cubic", 4), ("quadratic", 3)):
            f = getattr(L, "orc_find_roots_" + n)
            f.argtypes = [C.c_double] * k + [_D]
            f.restype = C.c_int
        L.orc_pattern_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                       C.POINTER(C.c_int64)]
        L.orc_get_inverse.argtypes = [C.c_void_p, C.c_int, _D]
        L.orc_intersect.argtypes = [C.c_void_p, _D, _D, C.c_int, _D, _I, _D, _D]
        L.orc_local_intersect.argtypes = [C.c_void_p, C.c_int, _D, _D, C.c_int, _D, _I, _D, _D]
        L.orc_color_at.argtypes = [C.c_void_p, _D, _D, C.c_int, _D]
        L.orc_shade.argtypes = [C.c_void_p, _D, _D, C.c_int, _D, _I, _D, _D, C.c_int, C.c_int, C.c_int, _D]
        L.orc_prepare_computations.argtypes = [C.c_void_p, _D, _D, C.c_int, _D, _I, _D, _D, C.c_int, _D]
        L.orc_is_shadowed.argtypes = [C.c_void_p, _D, _D]
        L.orc_lighting.argtypes = [C.c_void_p, C.c_int, C.c_int, _D, _D, _D, C.c_double, _D]
        L.orc_pattern_at.argtypes = [C.c_void_p, C.c_int, _D, _D]
        L.orc_normal_at.argtypes = [C.c_void_p, C.c_int, _D, C.c_double, C.c_double, _D]
        L.orc_world_to_object.argtypes = [C.c_void_p, C.c_int, _D, _D]
        L.orc_normal_to_world.argtypes = [C.c_void_p, C.c_int, _D, _D]
        L.orc_group_aabb.argtypes = [C.c_void_p, C.c_int, _D]
        L.orc_camera_new.argtypes = [C.c_int64, C.c_int64, C.c_double, _D, C.POINTER(OracleCamera)]
        L.orc_ray_for_pixel.argtypes = [C.POINTER(OracleCamera), C.c_int64, C.c_int64, _D, _D]
        L.orc_render.argtypes = [C.c_void_p, C.POINTER(OracleCamera), C.c_int, C.c_uint64, C.c_int, C.c_int,
                                 C.c_int, C.c_int, C.c_int, _D, C.POINTER(OrcStats)]
        L.orc_aa_average.argtypes = [_D, C.c_int64, C.c_int64, C.c_int, _D]
        L.orc_quantize.argtypes = [_D, C.c_int64, C.POINTER(C.c_uint8)]
        L.orc_jitter.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_jitter.restype = C.c_double
        L.orc_set_context.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint64]
        L.orc_set_pow_mode.argtypes = [C.c_void_p, C.c_int]
        L.orc_get_stats.argtypes = [C.c_void_p, C.POINTER(OrcStats)]
        L.orc_set_shape_params.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_int]
        L.orc_set_csg_op.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_csg_allowed.argtypes = [C.c_int] * 4
        L.orc_pattern_set_noise.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_double]
        L.orc_noise_3d.argtypes = [C.c_double] * 3
        L.orc_noise_3d.restype = C.c_double
        L.orc_octave_perlin.argtypes = [C.c_double] * 3 + [C.c_int64, C.c_double]
        L.orc_octave_perlin.restype = C.c_double
        L.orc_get_shape_params.argtypes = [C.c_void_p, C.c_int, _D]
        L.orc_get_csg_op.argtypes = [C.c_void_p, C.c_int]
        L.orc_csg_filter.argtypes = [C.c_void_p, C.c_int, C.c_int, _D, _I, _I]
        for n in ("orc_mat_identity",):
            getattr(L, n).argtypes = [_D]
        L.orc_mat_translate.argtypes = [C.c_double] * 3 + [_D]
        L.orc_mat_scale.argtypes = [C.c_double] * 3 + [_D]
        L.orc_mat_rotate.argtypes = [C.c_int, C.c_double, _D]
        L.orc_mat_shear.argtypes = [C.c_double] * 6 + [_D]
        L.orc_mat_multiply.argtypes = [_D, _D, _D]
        L.orc_mat_inverse.argtypes = [_D, _D]
        L.orc_mat_determinant.argtypes = [_D]
        L.orc_mat_determinant.restype = C.c_double
        L.orc_mat_view_transform.argtypes = [_D, _D, _D, _D]
        L.orc_mat_multiply_tuple.argtypes = [_D, _D, _D]
        _lib = L
    return _lib


def _dv(vals, n=None):
    vals = [float(x) for x in vals]
    arr = (C.c_double * (n or len(vals)))(*vals)
    return arr


def _out(n):
    return (C.c_double * n)()


class Mat:
    """4x4 matrix helpers computed by the oracle's restatement of matrix.rs."""

    @staticmethod
    def identity():
        o = _out(16)
        _load().orc_mat_identity(o)
        return list(o)

    @staticmethod
    def translate(x, y, z):
        o = _out(16)
        _load().orc_mat_translate(x, y, z, o)
        return list(o)

    @staticmethod
    def scale(x, y, z):
        o = _out(16)
        _load().orc_mat_scale(x, y, z, o)
        return list(o)

    @staticmethod
    def rotate(axis, radians):
        o = _out(16)
        _load().orc_mat_rotate({"x": 0, "y": 1, "z": 2}.get(axis, axis), radians, o)
        return list(o)

    @staticmethod
    def shear(*a):
        o = _out(16)
        _load().orc_mat_shear(*[float(x) for x in a], o)
        return list(o)

    @staticmethod
    def multiply(a, b):
        o = _out(16)
        _load().orc_mat_multiply(_dv(a), _dv(b), o)
        return list(o)

    @staticmethod
    def inverse(a):
        o = _out(16)
        _load().orc_mat_inverse(_dv(a), o)
        return list(o)

    @staticmethod
    def determinant(a):
        return _load().orc_mat_determinant(_dv(a))

    @staticmethod
    def view_transform(f, t, u):
        o = _out(16)
        _load().orc_mat_view_transform(_dv(f), _dv(t), _dv(u), o)
        return list(o)

    @staticmethod
    def multiply_tuple(m, t):
        o = _out(4)
        _load().orc_mat_multiply_tuple(_dv(m), _dv(t), o)
        return list(o)


DEFAULT_MAT7 = (0.1, 0.9, 0.9, 200.0, 0.0, 0.0, 1.0)  # material.rs:47-58

PAT = {"test": 0, "solid": 1, "stripe": 2, "gradient": 3, "ring": 4, "checker": 5, "blend": 6, "perturbed": 7,
       "noise": 8, "texture": 9}
KIND = {"sphere": 0, "plane": 1, "group": 2, "triangle": 3, "smooth_triangle": 4, "cube": 5, "cylinder": 6,
        "cone": 7, "csg": 8, "torus": 9}
CSG_OP = {"union": 0, "intersection": 1, "difference": 2}  # csg.rs:13-17


class Oracle:
    """One reference 'Scene' + its object registry (object/db.rs)."""

    mat = Mat

    def __init__(self):
        self.L = _load()
        self.w = C.c_void_p(self.L.orc_world_new())

    def __del__(self):
        try:
            if self.w:
                self.L.orc_world_free(self.w)
                self.w = None
        except Exception:
            pass

    # --- construction ---
    def add(self, kind, parent=-1, transform=None, material=None, pattern=-1):
        oid = self.L.orc_add_object(self.w, KIND[kind] if isinstance(kind, str) else kind, parent)
        if transform is not None:
            self.set_transform(oid, transform)
        if material is not None or pattern != -1:
            self.set_material(oid, material or DEFAULT_MAT7, pattern)
        return oid

    def set_shape_params(self, oid, minimum=-math.inf, maximum=math.inf, closed=False):
        """cylinder / cone: minimum, maximum, closed (cylinder.rs:29-37, cone.rs:30-38)"""
        self.L.orc_set_shape_params(self.w, oid, float(minimum), float(maximum), 1 if closed else 0)

    def add_csg(self, op, parent=-1, transform=None):
        """CSG; its left and right are the next two objects added with it as parent (csg.rs:51-65)."""
        oid = self.add("csg", parent, transform)
        self.L.orc_set_csg_op(self.w, oid, CSG_OP[op] if isinstance(op, str) else op)
        return oid

    def shape_params(self, oid):
        out = _out(3)
        self.L.orc_get_shape_params(self.w, oid, out)
        return list(out)

    def csg_op(self, oid):
        return self.L.orc_get_csg_op(self.w, oid)

    def csg_allowed(self, op, lhit, inl, inr):
        return bool(self.L.orc_csg_allowed(CSG_OP[op] if isinstance(op, str) else op, int(lhit), int(inl), int(inr)))

    def csg_filter(self, csg, xs):
        """xs: [(t, obj)] -> indices kept by filter_intersections (csg.rs:82-101)."""
        n = len(xs)
        keep = (C.c_int * max(n, 1))()
        k = self.L.orc_csg_filter(self.w, csg, n, _dv([x[0] for x in xs], max(n, 1)),
                                  (C.c_int * max(n, 1))(*[x[1] for x in xs]), keep)
        return [keep[i] for i in range(k)]

    def add_triangle(self, p1, p2, p3, parent=-1):
        return self.L.orc_add_triangle(self.w, parent, _dv(p1), _dv(p2), _dv(p3))

    def add_smooth_triangle(self, p1, p2, p3, n1, n2, n3, parent=-1):
        return self.L.orc_add_smooth_triangle(self.w, parent, _dv(p1), _dv(p2), _dv(p3), _dv(n1), _dv(n2), _dv(n3))

    def load_obj(self, path, parent=-1, material=DEFAULT_MAT7, pattern=-1):
        r = self.L.orc_load_obj(self.w, path.encode(), parent, _dv(material), pattern)
        if r < 0:
            raise RuntimeError(f"oracle OBJ load failed ({r}): {path}")
        return r

    def set_transform(self, oid, m):
        self.L.orc_set_transform(self.w, oid, _dv(m))

    def set_material(self, oid, mat7=DEFAULT_MAT7, pattern=-1):
        self.L.orc_set_material(self.w, oid, _dv(mat7), pattern)

    def pattern(self, kind, color=None, a=-1, b=-1, scale=0.5, transform=None):
        k = PAT[kind] if isinstance(kind, str) else kind
        return self.L.orc_pattern_new(self.w, k, _dv(color) if color is not None else None, a, b, float(scale),
                                      _dv(transform) if transform is not None else None)

    def set_noise(self, pid, octaves, persistence):
        self.L.orc_pattern_set_noise(self.w, pid, int(octaves), float(persistence))

    def point_light(self, pos, color):
        return self.L.orc_add_point_light(self.w, _dv(pos), _dv(color))

    def area_light(self, corner, u, v, color, level):
        return self.L.orc_add_area_light(self.w, _dv(corner), _dv(u), _dv(v), _dv(color), int(level))

    def remove_light(self, i):
        self.L.orc_remove_light(self.w, i)

    def num_children(self, oid):
        return self.L.orc_num_children(self.w, oid)

    def num_objects(self):
        return self.L.orc_num_objects(self.w)

    def add_texture(self, rgba):
        """rgba: (height, width, 4) uint8, rows top to bottom (texture.rs:15-19)."""
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        assert a.ndim == 3 and a.shape[2] == 4
        return self.L.orc_add_texture(self.w, a.shape[1], a.shape[0], a.ctypes.data_as(C.POINTER(C.c_uint8)))

    def texture_color(self, tex, u, v):
        out = (C.c_uint8 * 4)()
        self.L.orc_texture_color(self.w, tex, float(u), float(v), out)
        return list(out)

    def uv_mapping(self, oid, p):
        out = (C.c_double * 2)()
        self.L.orc_uv_mapping(self.w, oid, _dv(p), out)
        return out[0], out[1]

    @staticmethod
    def find_roots(*coeffs):
        """roots 0.0.8 find_roots_{quadratic,cubic,quartic} by the number of coefficients."""
        L = _load()
        f = {3: L.orc_find_roots_quadratic, 4: L.orc_find_roots_cubic, 5: L.orc_find_roots_quartic}[len(coeffs)]
        out = (C.c_double * 4)()
        n = f(*[float(c) for c in coeffs], out)
        return [out[i] for i in range(n)]

    def num_patterns(self):
        return self.L.orc_num_patterns(self.w)

    def pattern_info(self, pid):
        """(kind, a, b, scale, octaves, persistence) of one pattern tree node."""
        ints, dbl, octv = (C.c_int32 * 3)(), (C.c_double * 2)(), C.c_int64()
        self.L.orc_pattern_info(self.w, pid, ints, dbl, C.byref(octv))
        return ints[0], ints[1], ints[2], dbl[0], octv.value, dbl[1]

    def inverse_of(self, oid):
        o = _out(16)
        self.L.orc_get_inverse(self.w, oid, o)
        return list(o)

    def set_pow_mode(self, mode):
        """DIAGNOSTIC: 1 = correctly rounded x^n for integer shininess (libm pow is not always correctly
        rounded); 0 = std::pow as the reference (the default, and the parity reference)."""
        self.L.orc_set_pow_mode(self.w, int(mode))

    def set_context(self, seed=0, jitter_mode=0, sample=0):
        self.L.orc_set_context(self.w, seed, jitter_mode, sample)

    def stats(self):
        s = OrcStats()
        self.L.orc_get_stats(self.w, C.byref(s))
        return s.as_dict()

    # --- queries (reference unit-test entry points) ---
    def intersect(self, o, d, cap=4096):
        t, ob, u, v = _out(cap), (C.c_int * cap)(), _out(cap), _out(cap)
        n = self.L.orc_intersect(self.w, _dv(o), _dv(d), cap, t, ob, u, v)
        return [(t[i], ob[i], u[i], v[i]) for i in range(min(n, cap))]

    def local_intersect(self, oid, o4, d4, cap=4096):
        t, ob, u, v = _out(cap), (C.c_int * cap)(), _out(cap), _out(cap)
        n = self.L.orc_local_intersect(self.w, oid, _dv(o4), _dv(d4), cap, t, ob, u, v)
        return [(t[i], ob[i], u[i], v[i]) for i in range(min(n, cap))]

    def color_at(self, o, d, remaining=5):
        out = _out(3)
        self.L.orc_color_at(self.w, _dv(o), _dv(d), remaining, out)
        return tuple(out)

    def _xs(self, xs):
        n = len(xs)
        t = _dv([x[0] for x in xs], max(n, 1))
        ob = (C.c_int * max(n, 1))(*[x[1] for x in xs])
        u = _dv([x[2] if len(x) > 2 else 0.0 for x in xs], max(n, 1))
        v = _dv([x[3] if len(x) > 3 else 0.0 for x in xs], max(n, 1))
        return n, t, ob, u, v

    def shade(self, o, d, xs, hit, remaining=5, what="shade_hit"):
        n, t, ob, u, v = self._xs(xs)
        out = _out(3)
        self.L.orc_shade(self.w, _dv(o), _dv(d), n, t, ob, u, v, hit, remaining,
                         {"shade_hit": 0, "reflected": 1, "refracted": 2}[what], out)
        return tuple(out)

    def prepare_computations(self, o, d, xs, hit):
        n, t, ob, u, v = self._xs(xs)
        out = _out(27)
        self.L.orc_prepare_computations(self.w, _dv(o), _dv(d), n, t, ob, u, v, hit, out)
        r = list(out)
        return {"t": r[0], "point": r[1:5], "eyev": r[5:9], "normalv": r[9:13], "inside": bool(r[13]),
                "over_point": r[14:18], "under_point": r[18:22], "reflectv": r[22:25], "n1": r[25], "n2": r[26]}

    def is_shadowed(self, p, light_pos):
        return bool(self.L.orc_is_shadowed(self.w, _dv(p), _dv(light_pos)))

    def lighting(self, obj, light, point, eyev, normalv, in_shadow):
        out = _out(3)
        self.L.orc_lighting(self.w, obj, light, _dv(point), _dv(eyev), _dv(normalv), float(in_shadow), out)
        return tuple(out)

    def pattern_at(self, pattern, p):
        out = _out(3)
        self.L.orc_pattern_at(self.w, pattern, _dv(p), out)
        return tuple(out)

    def normal_at(self, obj, p, u=0.0, v=0.0):
        out = _out(4)
        self.L.orc_normal_at(self.w, obj, _dv(p), u, v, out)
        return tuple(out)

    def world_to_object(self, obj, p):
        out = _out(4)
        self.L.orc_world_to_object(self.w, obj, _dv(p), out)
        return tuple(out)

    def normal_to_world(self, obj, n):
        out = _out(4)
        self.L.orc_normal_to_world(self.w, obj, _dv(n), out)
        return tuple(out)

    def group_aabb(self, oid):
        out = _out(6)
        self.L.orc_group_aabb(self.w, oid, out)
        return tuple(out)

    # --- camera / render ---
    @staticmethod
    def camera(hsize, vsize, fov, transform=None):
        c = OracleCamera()
        _load().orc_camera_new(hsize, vsize, fov, _dv(transform) if transform is not None else None, C.byref(c))
        return c

    @staticmethod
    def ray_for_pixel(cam, px, py):
        o, d = _out(4), _out(4)
        _load().orc_ray_for_pixel(C.byref(cam), px, py, o, d)
        return tuple(o), tuple(d)

    def render(self, cam, max_depth=5, seed=0, jitter_mode=0, threads=0, band=1, band_stride=1, band_phase=0):
        """Supersampled canvas (vsize, hsize, 3) f64 + stats dict.  Unrendered rows are NaN."""
        canvas = np.full((cam.vsize, cam.hsize, 3), np.nan, dtype=np.float64)
        st = OrcStats()
        rc = self.L.orc_render(self.w, C.byref(cam), max_depth, seed, jitter_mode, threads, band, band_stride,
                               band_phase, canvas.ctypes.data_as(_D), C.byref(st))
        if rc != 0:
            raise RuntimeError("reference would panic: NaN intersection t in sort (scene.rs:104)")
        return canvas, st.as_dict()

    @staticmethod
    def aa_average(canvas, aa):
        vs, hs, _ = canvas.shape
        canvas = np.ascontiguousarray(canvas, dtype=np.float64)
        out = np.zeros((vs // aa, hs // aa, 3), dtype=np.float64)
        _load().orc_aa_average(canvas.ctypes.data_as(_D), hs, vs, aa, out.ctypes.data_as(_D))
        return out

    @staticmethod
    def quantize(avg):
        avg = np.ascontiguousarray(avg, dtype=np.float64)
        n = avg.shape[0] * avg.shape[1]
        out = np.zeros((avg.shape[0], avg.shape[1], 4), dtype=np.uint8)
        _load().orc_quantize(avg.ctypes.data_as(_D), n, out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out

    @staticmethod
    def jitter(seed, sample, path, light, s, which):
        return _load().orc_jitter(seed, sample, path, light, s, which)

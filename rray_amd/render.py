"""Host-side mirror of the reference's render-path interface over the C ABI.

Reference names kept where they exist:
  Scene::add_light / add_object, Sphere::new, Plane::new, Group::add_child  -> SceneBuilder
  Camera::new (camera.rs:41) / Camera::render (camera.rs:107)               -> camera(), Renderer.render
  Scene::color_at (scene.rs:128), Scene::is_shadowed (scene.rs:234)         -> Renderer.color_at / is_shadowed
  render_scene_from_str / render_scene_from_file (scene_builder_yaml.rs:387,429)
Every call goes to librray_amd.so's HIP kernels; there is no CPU path.
"""
import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import check, lib

DEFAULT_MATERIAL = (0.1, 0.9, 0.9, 200.0, 0.0, 0.0, 1.0)  # material.rs:47-58
IDENTITY = tuple(float(i == j) for i in range(4) for j in range(4))


def _dp(a):
    return a.ctypes.data_as(_lib._D)


def _ip(a):
    return a.ctypes.data_as(_lib._I)


class SceneBuilder:
    """Programmatic scene with the reference's registry semantics (object/db.rs, scene.rs:24-71)."""

    def __init__(self):
        self.kind, self.parent, self.material, self.transform, self.tri, self.kids, self.top = [], [], [], [], [], [], []
        self.mats, self.mat_pattern = [], []
        self.pat_kind, self.pat_a, self.pat_b, self.pat_color, self.pat_scale, self.pat_transform = [], [], [], [], [], []
        self.pat_octaves, self.pat_persistence = [], []
        self.textures = []  # (height, width, 4) uint8 RGBA arrays
        self.light_kind, self.light, self.light_level = [], [], []
        self.shape, self.csg_op = [], []
        self._keep = None

    # --- materials / patterns (material.rs, pattern.rs)
    def pattern(self, kind, color=(0.0, 0.0, 0.0), a=-1, b=-1, scale=0.5, transform=IDENTITY, octaves=1,
                persistence=1.0):
        """A pattern tree node (pattern.rs:23-27); octaves / persistence are Perturbed / Noise's."""
        self.pat_kind.append(_lib.PAT[kind] if isinstance(kind, str) else int(kind))
        self.pat_a.append(a)
        self.pat_b.append(b)
        self.pat_color.extend(float(x) for x in color)
        self.pat_scale.append(float(scale))
        self.pat_transform.extend(float(x) for x in transform)
        self.pat_octaves.append(int(octaves))
        self.pat_persistence.append(float(persistence))
        return len(self.pat_kind) - 1

    def texture(self, rgba):
        """Register an RGBA8 image (rows top to bottom, texture.rs:15-19); returns its index for
        pattern("texture", a=index)."""
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        if a.ndim != 3 or a.shape[2] != 4 or a.shape[0] < 1 or a.shape[1] < 1:
            raise ValueError("texture must be a non-empty (height, width, 4) uint8 array")
        self.textures.append(a)
        return len(self.textures) - 1

    def new_material(self, mat7=DEFAULT_MATERIAL, pattern=-1):
        self.mats.extend(float(x) for x in mat7)
        self.mat_pattern.append(pattern)
        return len(self.mat_pattern) - 1

    # --- objects
    def _obj(self, kind, parent, transform, material, pattern, tri=None):
        oid = len(self.kind)
        self.kind.append(kind)
        self.parent.append(parent)
        if kind in (_lib.GROUP, _lib.CSG):
            self.material.append(-1)
        else:
            self.material.append(material if isinstance(material, int) else self.new_material(
                material or DEFAULT_MATERIAL, pattern))
        self.transform.extend(float(x) for x in (transform or IDENTITY))
        self.tri.extend([float(x) for x in tri] if tri is not None else [0.0] * 18)
        self.kids.append([])
        self.shape.extend([-math.inf, math.inf, 0.0])
        self.csg_op.append(0)
        (self.kids[parent] if parent >= 0 else self.top).append(oid)
        return oid

    def sphere(self, transform=None, material=None, pattern=-1, parent=-1):
        return self._obj(_lib.SPHERE, parent, transform, material, pattern)

    def plane(self, transform=None, material=None, pattern=-1, parent=-1):
        return self._obj(_lib.PLANE, parent, transform, material, pattern)

    def group(self, transform=None, parent=-1):
        return self._obj(_lib.GROUP, parent, transform, None, -1)

    def cube(self, transform=None, material=None, pattern=-1, parent=-1):
        return self._obj(_lib.CUBE, parent, transform, material, pattern)

    def cylinder(self, minimum=-math.inf, maximum=math.inf, closed=False, transform=None, material=None, pattern=-1,
                 parent=-1, cone=False):
        oid = self._obj(_lib.CONE if cone else _lib.CYLINDER, parent, transform, material, pattern)
        self.shape[3 * oid:3 * oid + 3] = [float(minimum), float(maximum), 1.0 if closed else 0.0]
        return oid

    def cone(self, minimum=-math.inf, maximum=math.inf, closed=False, transform=None, material=None, pattern=-1,
             parent=-1):
        return self.cylinder(minimum, maximum, closed, transform, material, pattern, parent, cone=True)

    def csg(self, op, transform=None, parent=-1):
        """CSG node; add its left then its right child with parent=<this id> (csg.rs:51-65)."""
        oid = self._obj(_lib.CSG, parent, transform, None, -1)
        self.csg_op[oid] = _lib.CSG_OPS[op] if isinstance(op, str) else int(op)
        return oid

    def torus(self, minor_radius, transform=None, material=None, pattern=-1, parent=-1):
        """Torus in the xy plane, major radius 1 (torus.rs:23-31)."""
        oid = self._obj(_lib.TORUS, parent, transform, material, pattern)
        self.shape[3 * oid] = float(minor_radius)
        return oid

    def triangle(self, p1, p2, p3, transform=None, material=None, pattern=-1, parent=-1):
        return self._obj(_lib.TRIANGLE, parent, transform, material, pattern, list(p1) + list(p2) + list(p3) + [0.0] * 9)

    def smooth_triangle(self, p1, p2, p3, n1, n2, n3, transform=None, material=None, pattern=-1, parent=-1):
        return self._obj(_lib.SMOOTH_TRIANGLE, parent, transform, material, pattern,
                         list(p1) + list(p2) + list(p3) + list(n1) + list(n2) + list(n3))

    # --- lights (light.rs:37-45)
    def point_light(self, position, intensity):
        self.light_kind.append(_lib.LIGHT_POINT)
        self.light_level.append(0)
        self.light.extend([float(x) for x in position] + [float(x) for x in intensity] + [0.0] * 9)
        return len(self.light_kind) - 1

    def area_light(self, corner, u, v, intensity, level):
        c, u, v = [float(x) for x in corner], [float(x) for x in u], [float(x) for x in v]
        center = [(c[k] + u[k] * 0.5) + v[k] * 0.5 for k in range(3)]  # Python floats == f64 ops
        self.light_kind.append(_lib.LIGHT_AREA)
        self.light_level.append(int(level))
        self.light.extend(center + [float(x) for x in intensity] + c + u + v)
        return len(self.light_kind) - 1

    def desc(self):
        child_start, child_count, children = [], [], []
        for ks in self.kids:
            child_start.append(len(children))
            child_count.append(len(ks))
            children.extend(ks)
        arr = {
            "kind": np.array(self.kind, np.int32), "parent": np.array(self.parent, np.int32),
            "transform": np.array(self.transform, np.float64), "material": np.array(self.material, np.int32),
            "tri": np.array(self.tri, np.float64), "child_start": np.array(child_start, np.int32),
            "child_count": np.array(child_count, np.int32), "children": np.array(children or [0], np.int32),
            "top": np.array(self.top or [0], np.int32), "mat": np.array(self.mats or [0.0], np.float64),
            "mat_pattern": np.array(self.mat_pattern or [0], np.int32),
            "pat_kind": np.array(self.pat_kind or [0], np.int32), "pat_a": np.array(self.pat_a or [0], np.int32),
            "pat_b": np.array(self.pat_b or [0], np.int32), "pat_color": np.array(self.pat_color or [0.0], np.float64),
            "pat_scale": np.array(self.pat_scale or [0.0], np.float64),
            "pat_transform": np.array(self.pat_transform or [0.0], np.float64),
            "light_kind": np.array(self.light_kind or [0], np.int32),
            "light": np.array(self.light or [0.0], np.float64),
            "light_level": np.array(self.light_level or [0], np.int32),
            "shape": np.array(self.shape or [0.0], np.float64), "csg_op": np.array(self.csg_op or [0], np.int32),
            "pat_octaves": np.array(self.pat_octaves or [0], np.int32),
            "pat_persistence": np.array(self.pat_persistence or [0.0], np.float64),
        }
        tex_size = [v for t in self.textures for v in (t.shape[1], t.shape[0])]
        texels = np.concatenate([t.reshape(-1) for t in self.textures]) if self.textures else np.zeros(4, np.uint8)
        arr["tex_size"] = np.array(tex_size or [0], np.int32)
        arr["texels"] = texels
        d = _lib.SceneDesc()
        d.n_objects = len(self.kind)
        d.n_top = len(self.top)
        d.n_materials = len(self.mat_pattern)
        d.n_patterns = len(self.pat_kind)
        d.n_lights = len(self.light_kind)
        d.n_textures = len(self.textures)
        for k, v in arr.items():
            if v.dtype == np.uint8:
                setattr(d, k, v.ctypes.data_as(C.POINTER(C.c_uint8)))
            else:
                setattr(d, k, _dp(v) if v.dtype == np.float64 else _ip(v))
        d.inverse = None
        self._keep = arr
        return d


class YamlScene:
    """Product front-end: scene_builder_yaml.rs restated in C++ (rr_scene_from_yaml)."""

    def __init__(self, text, width, height, aa=1, obj_root=None):
        h = C.c_void_p()
        cam = _lib.Camera()
        check(lib().rr_scene_from_yaml(text.encode(), obj_root.encode() if obj_root else None, width, height, aa,
                                       C.byref(h), C.byref(cam)))
        self.h, self.camera, self.width, self.height, self.aa = h, cam, width, height, aa

    def desc(self):
        return lib().rr_scene_desc_of(self.h).contents

    def __del__(self):
        try:
            if self.h:
                lib().rr_scene_free(self.h)
                self.h = None
        except Exception:
            pass


def camera(hsize, vsize, field_of_view, transform=None):
    """Camera::new (camera.rs:41-63); sizes are the supersampled W*aa x H*aa."""
    cam = _lib.Camera()
    t = (C.c_double * 16)(*(transform or IDENTITY))
    check(lib().rr_camera_new(hsize, vsize, field_of_view, t, C.byref(cam)))
    return cam


def part_rows(height, part, nparts, block_rows=8):
    n = lib().rr_part_rows(height, part, nparts, block_rows, None)
    if n < 0:
        check(int(n))
    out = np.zeros(max(n, 1), np.int64)
    lib().rr_part_rows(height, part, nparts, block_rows, out.ctypes.data_as(C.POINTER(C.c_int64)))
    return out[:n]


def stage_row_offset(height, part, nparts, block_rows=8):
    """rr_stage_row_offset: first row of part `part`'s tile in the staging buffer (the rows of parts below it)."""
    n = lib().rr_stage_row_offset(height, part, nparts, block_rows)
    if n < 0:
        check(int(n))
    return int(n)


def unshuffle(staged, height, nparts, block_rows=8):
    """rr_unshuffle_host: the root's un-interleave on the host.  staged: (height, W, 3) f64, the parts' tiles back to
    back and unpadded, part p's rows at stage_row_offset(height, p, nparts, block_rows) — the staging buffer the
    library's per-part receives fill on rank 0 (multi.cpp)."""
    g = np.ascontiguousarray(staged, np.float64)
    if nparts < 1 or block_rows < 1 or height < 0:
        raise ValueError(f"unshuffle: bad partition (height {height}, nparts {nparts}, block_rows {block_rows})")
    # the library reads height rows of W * 3 doubles: refuse any other buffer before it does
    if g.ndim != 3 or g.shape[0] != height or g.shape[2] != 3:
        raise ValueError(f"unshuffle: staged must have shape ({height}, W, 3) for height {height}; got {g.shape}")
    W = g.shape[1]
    frame = np.zeros((height, W, 3), np.float64)
    check(lib().rr_unshuffle_host(_dp(g), _dp(frame), W, height, nparts, block_rows))
    return frame


def balance_bands(row_cost, nparts, root_extra=0.0, align=8):
    """rr_balance_bands: band bounds (nparts + 1) over len(row_cost) rows with even cost per band, part 0 carrying
    root_extra on top, inner bounds multiples of align."""
    c = np.ascontiguousarray(row_cost, np.float64)
    out = np.zeros(nparts + 1, np.int64)
    check(lib().rr_balance_bands(_dp(c), len(c), nparts, float(root_extra), align,
                                 out.ctypes.data_as(C.POINTER(C.c_int64))))
    return out


def device_count():
    n = C.c_int(0)
    lib().rr_device_count(C.byref(n))
    return n.value


def rccl_unique_id():
    """rr_rccl_unique_id: the bytes rank 0 shares with the other ranks before Renderer.rank(...)."""
    buf = (C.c_uint8 * _lib.RCCL_ID_BYTES)()
    check(lib().rr_rccl_unique_id(buf, _lib.RCCL_ID_BYTES))
    return bytes(buf)


class Renderer:
    """A gfx950 render context (rr_ctx): scene in HBM + the wavefront kernels.  Renderer(d) drives one
    device; Renderer.multi(ids) several devices of this process, Renderer.rank(d, n, r, uid) one rank of
    a one-process-per-GPU group — both split each frame in row tiles and gather them with RCCL."""

    def __init__(self, device=0, _handle=None):
        self.h = C.c_void_p()
        if _handle is not None:
            self.h = _handle
        else:
            check(lib().rr_create(device, C.byref(self.h)))
        self.device = device

    @classmethod
    def multi(cls, device_ids):
        ids = (C.c_int * len(device_ids))(*device_ids)
        h = C.c_void_p()
        check(lib().rr_create_multi(len(device_ids), ids, C.byref(h)))
        return cls(device_ids[0], _handle=h)

    @classmethod
    def rank(cls, device, nranks, rank, unique_id):
        uid = (C.c_uint8 * _lib.RCCL_ID_BYTES).from_buffer_copy(unique_id)
        h = C.c_void_p()
        check(lib().rr_create_rank(device, nranks, rank, uid, C.byref(h)))
        return cls(device, _handle=h)

    @classmethod
    def virtual(cls, device, nparts):
        """rr_create_virtual: nparts virtual ranks on one device (the multi-GPU frame assembly with the
        RCCL transfer replaced by device-local copies)."""
        h = C.c_void_p()
        check(lib().rr_create_virtual(device, nparts, C.byref(h)))
        return cls(device, _handle=h)

    def info(self):
        """(nranks, first global rank of this context, local devices)."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().rr_context_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def render_gather_device(self, cam, opts, d_frame, stream=None):
        """Whole frame (row tiles over the group's devices + one RCCL send / receive per part) into d_frame on rank 0's
        device, in `stream` order (asynchronous)."""
        check(lib().rr_render_gather_device(self.h, C.byref(cam), C.byref(opts), C.c_void_p(d_frame) if d_frame else None,
                                            C.c_void_p(stream) if stream else None))

    def bands(self):
        """rr_group_bands: the band bounds of a multi-device context (nranks + 1 rows), or None before its first
        band frame calibrated them."""
        nranks = self.info()[0]
        out = (C.c_int64 * (nranks + 1))()
        n = lib().rr_group_bands(self.h, out, nranks + 1)
        if n < 0:
            check(n)
        return list(out) if n else None

    def set_bands(self, bounds):
        """rr_group_set_bands: impose the band bounds (every rank the same)."""
        b = (C.c_int64 * len(bounds))(*bounds)
        check(lib().rr_group_set_bands(self.h, b, len(bounds)))

    def close(self):
        if getattr(self, "h", None):
            lib().rr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene):
        d = scene.desc()
        check(lib().rr_scene_upload(self.h, C.byref(d)))
        self._scene = scene

    def render(self, cam, aa=1, max_depth=5, seed=0, jitter_mode=0, part=0, nparts=1, block_rows=8, canvas=False,
               avg=True, band=None, interleave=False):
        """Camera::render -> dict(avg=(rows, W, 3) f64 before `as u8`, canvas=(rows*aa, W*aa, 3), stats).
        band=(row_begin, row_end): only those output rows (ABI 10); interleave: a multi-device context splits the
        frame in interleaved tiles (RR_PART_INTERLEAVE) instead of cost-balanced bands."""
        o = _lib.RenderOpts(aa, max_depth, seed, jitter_mode, part, nparts, block_rows,
                            (_lib.RR_OUT_CANVAS if canvas else 0) | (_lib.RR_OUT_AVG if avg else 0) |
                            (_lib.RR_PART_INTERLEAVE if interleave else 0), *(band or (0, 0)))
        H, W = cam.vsize // aa, cam.hsize // aa
        rows = max(band[1] - band[0], 0) if band else len(part_rows(H, part, nparts, block_rows))
        out_avg = np.zeros((rows, W, 3), np.float64) if avg else None
        out_canvas = np.zeros((rows * aa, cam.hsize, 3), np.float64) if canvas else None
        st = _lib.Stats()
        check(lib().rr_render(self.h, C.byref(cam), C.byref(o), _dp(out_canvas) if canvas else None,
                              _dp(out_avg) if avg else None, C.byref(st)))
        return {"avg": out_avg, "canvas": out_canvas, "stats": st.as_dict()}

    def render_device(self, cam, opts, d_canvas, d_avg, stream=None):
        """Renders into device buffers (ints: device pointers), ordered on `stream` (int or None)."""
        check(lib().rr_render_device(self.h, C.byref(cam), C.byref(opts), C.c_void_p(d_canvas or 0) if d_canvas else None,
                                     C.c_void_p(d_avg) if d_avg else None, C.c_void_p(stream) if stream else None))

    def kernel_profile(self, enable=True):
        check(lib().rr_kernel_profile(self.h, 1 if enable else 0))

    def kernel_times(self):
        """{kernel: (total_ms, launches)} accumulated since kernel_profile(True)."""
        ms = (C.c_double * 16)()
        n = (C.c_uint64 * 16)()
        k = lib().rr_kernel_times(self.h, ms, n, 16)
        if k < 0:
            check(k)
        return {_lib.KERNELS[i]: (ms[i], int(n[i])) for i in range(k)}

    def last_stats(self):
        st = _lib.Stats()
        check(lib().rr_last_stats(self.h, C.byref(st)))
        return st.as_dict()

    def color_at(self, origins, directions, remaining=5, seed=0, jitter_mode=0):
        o = np.ascontiguousarray(origins, np.float64).reshape(-1, 3)
        d = np.ascontiguousarray(directions, np.float64).reshape(-1, 3)
        out = np.zeros_like(o)
        check(lib().rr_color_at(self.h, len(o), _dp(o), _dp(d), remaining, seed, jitter_mode, _dp(out)))
        return out

    def is_shadowed(self, points, light_positions):
        p = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
        lp = np.ascontiguousarray(light_positions, np.float64).reshape(-1, 3)
        out = np.zeros(len(p), np.int32)
        check(lib().rr_is_shadowed(self.h, len(p), _dp(p), _dp(lp), _ip(out)))
        return out.astype(bool)


def quantize(avg):
    """canvas.rs:97-100: `(v*255.0) as u8` per channel + alpha 255."""
    avg = np.ascontiguousarray(avg, np.float64)
    n = avg.shape[0] * avg.shape[1]
    out = np.zeros((avg.shape[0], avg.shape[1], 4), np.uint8)
    check(lib().rr_quantize(_dp(avg), n, out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def write_png(path, rgba):
    rgba = np.ascontiguousarray(rgba, np.uint8)
    check(lib().rr_write_png(path.encode(), rgba.ctypes.data_as(C.POINTER(C.c_uint8)), rgba.shape[1], rgba.shape[0]))


def render_scene_from_str(text, width, height, png_file, aa=1, device=0, obj_root=None):
    """scene_builder_yaml.rs:387-410 on the GPU."""
    s = YamlScene(text, width, height, aa, obj_root)
    r = Renderer(device)
    r.upload(s)
    res = r.render(s.camera, aa=aa)
    write_png(png_file, quantize(res["avg"]))
    return res


def render_scene_from_file(path, width, height, png_file, aa=1, device=0, devices=None):
    """scene_builder_yaml.rs:429-436 on the GPU (same error as the reference for a missing file);
    devices=[...] splits the frame over several GPUs (rr_create_multi)."""
    if devices:
        ids = (C.c_int * len(devices))(*devices)
        check(lib().rr_render_scene_from_file_devices(path.encode(), width, height, png_file.encode(), aa, len(devices),
                                                      ids))
        return
    check(lib().rr_render_scene_from_file(path.encode(), width, height, png_file.encode(), aa, device))

"""ctypes binding of librray_amd.so (include/rray/rray.h).

Loading fails loudly when the in-tree library is missing: there is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "librray_amd.so")
# Experiment builds (build.build_variant -> abtest/<name>/librray_amd.so) stand in for the product only
# when explicitly marked as an experiment run (RRAY_EXPERIMENT=1) and only from the repo's abtest/ tree;
# the product path always loads the in-tree library.
if os.environ.get("RRAY_LIB") and os.environ.get("RRAY_EXPERIMENT") == "1":
    _cand = os.path.realpath(os.environ["RRAY_LIB"])
    if not _cand.startswith(os.path.join(os.path.dirname(HERE), "abtest") + os.sep):
        raise RuntimeError(f"RRAY_LIB={_cand}: experiment libraries must live under abtest/")
    LIB_PATH = _cand
HEADER = os.path.join(os.path.dirname(HERE), "include", "rray", "rray.h")

RR_OK = 0
ERRORS = {-1: "RR_E_ARG", -2: "RR_E_HIP", -3: "RR_E_SCENE", -4: "RR_E_NONAFFINE", -5: "RR_E_LIMIT", -6: "RR_E_IO",
          -7: "RR_E_NAN"}
globals().update({name: code for code, name in ERRORS.items()})  # RR_E_ARG = -1, ...
RR_OUT_CANVAS, RR_OUT_AVG, RR_OUT_AVG_F32 = 1, 2, 4
RR_NO_FRAME_TIMING = 8  # rr_render_device: no per-frame HIP event pair (rr_stats.kernel_ms = 0)
RR_PART_INTERLEAVE = 16  # multi-device contexts: interleaved tiles + staging buffer + placement (ABI 9) instead of bands
SPHERE, PLANE, GROUP, TRIANGLE, SMOOTH_TRIANGLE, CUBE, CYLINDER, CONE, CSG, TORUS = range(10)
CSG_OPS = {"union": 0, "intersection": 1, "difference": 2}
PAT = {"test": 0, "solid": 1, "stripe": 2, "gradient": 3, "ring": 4, "checker": 5, "blend": 6, "perturbed": 7,
       "noise": 8, "texture": 9}
LIGHT_POINT, LIGHT_AREA = 0, 1
KERNELS = ["trace", "n1n2", "shade", "shadow", "finish", "combine", "aa", "trace_shade", "chain", "deep"]

_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int32)


class SceneDesc(C.Structure):
    _fields_ = [("n_objects", C.c_int32), ("kind", _I), ("parent", _I), ("transform", _D), ("inverse", _D),
                ("material", _I), ("tri", _D), ("child_start", _I), ("child_count", _I), ("children", _I),
                ("n_top", C.c_int32), ("top", _I), ("n_materials", C.c_int32), ("mat", _D), ("mat_pattern", _I),
                ("n_patterns", C.c_int32), ("pat_kind", _I), ("pat_a", _I), ("pat_b", _I), ("pat_color", _D),
                ("pat_scale", _D), ("pat_transform", _D), ("n_lights", C.c_int32), ("light_kind", _I),
                ("light", _D), ("light_level", _I), ("shape", _D), ("csg_op", _I), ("pat_octaves", _I),
                ("pat_persistence", _D), ("n_textures", C.c_int32), ("tex_size", _I),
                ("texels", C.POINTER(C.c_uint8))]


class Camera(C.Structure):
    _fields_ = [("hsize", C.c_int64), ("vsize", C.c_int64), ("field_of_view", C.c_double),
                ("pixel_size", C.c_double), ("half_width", C.c_double), ("half_height", C.c_double),
                ("transform", C.c_double * 16)]


class RenderOpts(C.Structure):
    _fields_ = [("aa", C.c_int32), ("max_depth", C.c_int32), ("seed", C.c_uint64), ("jitter_mode", C.c_int32),
                ("part", C.c_int32), ("nparts", C.c_int32), ("block_rows", C.c_int32), ("flags", C.c_int32),
                ("row_begin", C.c_int32), ("row_end", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("shade_events", C.c_uint64),
                ("n1n2_scans", C.c_uint64), ("group_tests", C.c_uint64), ("group_hits", C.c_uint64),
                ("samples", C.c_uint64), ("prim_tests", C.c_uint64), ("kernel_ms", C.c_double),
                ("exact_flops", C.c_uint64 * 3), ("wave_visits", C.c_uint64 * 3), ("nan_rays", C.c_uint64)]

    def as_dict(self):
        out = {}
        for n, _ in self._fields_:
            v = getattr(self, n)
            out[n] = list(v) if isinstance(v, C.Array) else v
        return out


EXPORTS = ["rr_abi_version", "rr_last_error", "rr_device_count", "rr_create", "rr_destroy", "rr_scene_upload",
           "rr_camera_new", "rr_render", "rr_render_device", "rr_part_rows", "rr_kernel_profile", "rr_kernel_times",
           "rr_last_stats", "rr_color_at",
           "rr_is_shadowed", "rr_scene_inspect", "rr_scene_from_yaml", "rr_scene_desc_of", "rr_scene_free", "rr_quantize",
           "rr_write_png", "rr_render_scene_from_file", "rr_render_scene_from_file_devices", "rr_create_multi",
           "rr_rccl_unique_id", "rr_create_rank", "rr_context_info", "rr_render_gather_device", "rr_create_virtual",
           "rr_unshuffle_host", "rr_stage_row_offset", "rr_build_digest", "rr_balance_bands", "rr_group_bands",
           "rr_group_set_bands"]
RCCL_ID_BYTES = 128

_lib = None


class RRError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    """The loaded library; raises when the HIP build is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    L.rr_abi_version.restype = C.c_int32
    L.rr_last_error.restype = C.c_char_p
    L.rr_device_count.argtypes = [C.POINTER(C.c_int)]
    L.rr_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.rr_destroy.argtypes = [C.c_void_p]
    L.rr_scene_upload.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    L.rr_camera_new.argtypes = [C.c_int64, C.c_int64, C.c_double, _D, C.POINTER(Camera)]
    L.rr_render.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(RenderOpts), _D, _D, C.POINTER(Stats)]
    L.rr_render_device.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(RenderOpts), C.c_void_p, C.c_void_p,
                                   C.c_void_p]
    L.rr_part_rows.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int64)]
    L.rr_part_rows.restype = C.c_int64
    L.rr_kernel_profile.argtypes = [C.c_void_p, C.c_int]
    L.rr_kernel_times.argtypes = [C.c_void_p, _D, C.POINTER(C.c_uint64), C.c_int32]
    L.rr_last_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    L.rr_color_at.argtypes = [C.c_void_p, C.c_int64, _D, _D, C.c_int32, C.c_uint64, C.c_int32, _D]
    L.rr_is_shadowed.argtypes = [C.c_void_p, C.c_int64, _D, _D, _I]
    L.rr_scene_inspect.argtypes = [C.POINTER(SceneDesc), _D, _D, _I]
    L.rr_scene_from_yaml.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int64, C.c_int32, C.POINTER(C.c_void_p),
                                     C.POINTER(Camera)]
    L.rr_scene_desc_of.argtypes = [C.c_void_p]
    L.rr_scene_desc_of.restype = C.POINTER(SceneDesc)
    L.rr_scene_free.argtypes = [C.c_void_p]
    L.rr_quantize.argtypes = [_D, C.c_int64, C.POINTER(C.c_uint8)]
    L.rr_write_png.argtypes = [C.c_char_p, C.POINTER(C.c_uint8), C.c_int64, C.c_int64]
    L.rr_render_scene_from_file.argtypes = [C.c_char_p, C.c_int64, C.c_int64, C.c_char_p, C.c_int32, C.c_int]
    L.rr_render_scene_from_file_devices.argtypes = [C.c_char_p, C.c_int64, C.c_int64, C.c_char_p, C.c_int32, C.c_int,
                                                    C.POINTER(C.c_int)]
    L.rr_create_multi.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p)]
    L.rr_rccl_unique_id.argtypes = [C.POINTER(C.c_uint8), C.c_int32]
    L.rr_create_rank.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_void_p)]
    L.rr_context_info.argtypes = [C.c_void_p, _I, _I, _I]
    L.rr_create_virtual.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.rr_unshuffle_host.argtypes = [_D, _D, C.c_int64, C.c_int64, C.c_int32, C.c_int32]
    L.rr_stage_row_offset.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    L.rr_stage_row_offset.restype = C.c_int64
    L.rr_render_gather_device.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(RenderOpts), C.c_void_p,
                                          C.c_void_p]
    L.rr_build_digest.restype = C.c_char_p
    L.rr_balance_bands.argtypes = [_D, C.c_int64, C.c_int32, C.c_double, C.c_int32, C.POINTER(C.c_int64)]
    L.rr_group_bands.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]
    L.rr_group_set_bands.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]
    _lib = L
    return L


def build_digest():
    """The source digest baked into the loaded library (rr_build_digest)."""
    return lib().rr_build_digest().decode()


def check_provenance():
    """(library digest, source digest) — raises when the loaded librray_amd.so was not built from the sources of
    this tree (a stale prebuilt library)."""
    from . import build

    have, want = build_digest(), build.source_digest()
    if have.startswith("variant-") and LIB_PATH != os.path.join(HERE, "_lib", "librray_amd.so"):
        return have, want  # an explicitly selected experiment build (RRAY_EXPERIMENT=1, abtest/): reported as such
    if have != want:
        raise RuntimeError(f"{LIB_PATH} was built from sources {have}, but this tree's sources are {want}: rebuild it "
                           "(python -c 'import __graft_entry__ as g; g.build()')")
    return have, want


def check(rc):
    if rc != RR_OK:
        raise RRError(rc, lib().rr_last_error().decode(errors="replace"))
    return rc

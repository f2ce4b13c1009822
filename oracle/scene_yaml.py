"""Restatement of scene_builder_yaml.rs (reference src/raytracer/scene_builder_yaml.rs:1-436)
over PyYAML, building an oracle world — TEST INFRASTRUCTURE ONLY.

PyYAML is an independent parser from the product's C++ YAML front-end; scalars are
re-typed here with yaml-rust2 0.8 rules (Yaml::from_str: i64 first, then f64, "true"/
"false", "~"/"null"; quoted scalars stay strings), because PyYAML's YAML-1.1 resolver
differs (e.g. "1e-5" is a string there, "010" octal).
"""
import math
import os
import re

import numpy as np
import yaml

from .oracle import DEFAULT_MAT7, Mat, Oracle

_RUST_FLOAT = re.compile(r"^[+-]?(inf|infinity|nan|(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))([eE][+-]?[0-9]+)?)$", re.I)
_RUST_INT = re.compile(r"^[+-]?[0-9]+$")


class Real(float):
    """yaml-rust2 Yaml::Real (kept distinct from Integer for as_i64 semantics)."""


def _plain(v):
    # yaml-rust2 Yaml::from_str
    if v.startswith("0x"):
        try:
            return int(v[2:], 16)
        except ValueError:
            pass
    elif v.startswith("0o"):
        try:
            return int(v[2:], 8)
        except ValueError:
            pass
    if v in ("~", "null"):
        return None
    if v == "true":
        return True
    if v == "false":
        return False
    if _RUST_INT.match(v):
        iv = int(v)
        if -(2**63) <= iv < 2**63:
            return iv
    if v in (".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf", "-.Inf", "-.INF", ".nan", ".NaN", ".NAN"):
        return ("badreal", v)  # Real whose later str::parse::<f64> would panic
    if _RUST_FLOAT.match(v):
        return Real(float(v))
    return v


class _Loader(yaml.SafeLoader):
    pass


_Loader.yaml_implicit_resolvers = {}


def _construct_str(loader, node):
    v = loader.construct_scalar(node)
    return _plain(v) if node.style is None else v


_Loader.add_constructor("tag:yaml.org,2002:str", _construct_str)

BAD = object()  # Yaml::BadValue


def _get(node, key):
    if isinstance(node, dict) and key in node:
        return node[key]
    return BAD


def get_f64(node):  # scene_builder_yaml.rs:68-74
    if isinstance(node, bool) or node is None or node is BAD or isinstance(node, (str, list, dict, tuple)):
        raise ValueError(f"{node!r} not a number")
    return float(node)


def get_f64_default(node, default):  # :76-82
    if isinstance(node, bool) or node is None or node is BAD or isinstance(node, (str, list, dict, tuple)):
        return default
    return float(node)


def _as_usize(v):  # Rust `f64 as usize`: truncate, saturate at 0, NaN -> 0
    if v != v or v <= 0:
        return 0
    return int(min(v, 2.0 ** 63))


def deg2rad(d):  # :25-27
    return d * math.pi / 180.0


def create_matrix(t):  # :178-216
    ty = _get(t, "type")
    if ty == "translate":
        a = _get(t, "amount")
        return Mat.translate(get_f64(a[0]), get_f64(a[1]), get_f64(a[2]))
    if ty == "scale":
        a = _get(t, "amount")
        return Mat.scale(get_f64(a[0]), get_f64(a[1]), get_f64(a[2]))
    if ty == "rotate":
        ang = deg2rad(get_f64(_get(t, "angle")))
        axis = _get(t, "axis")
        if axis not in ("x", "y", "z"):
            raise ValueError(f"Unknown axis: {axis}")
        return Mat.rotate(axis, ang)
    if ty == "shear":
        return Mat.shear(*[get_f64(_get(t, k)) for k in ("xy", "xz", "yx", "yz", "zx", "zy")])
    raise ValueError(f"Unknown transform type: {ty}")


def create_transforms(ts):  # :218-224 — reversed, m = m * T
    m = Mat.identity()
    if not isinstance(ts, list):
        ts = []
    for t in reversed(ts):
        m = Mat.multiply(m, create_matrix(t))
    return m


class YamlSceneBuilder:
    def __init__(self, orc: Oracle, obj_root=None):
        self.o = orc
        self.obj_root = obj_root
        self.textures = {}  # decoded image per path (each Pattern::texture holds its own copy)

    def color(self, v):
        return (get_f64(v[0]), get_f64(v[1]), get_f64(v[2]))

    def create_pattern(self, p):  # :226-308
        ts = _get(p, "transforms")
        transform = create_transforms(ts if isinstance(ts, list) else [])
        ty = _get(p, "type")
        if not isinstance(ty, str):
            raise ValueError("pattern type not found")
        color = _get(p, "color")
        color = [0.0, 0.0, 0.0] if color is BAD else color
        if ty == "solid":
            return self.o.pattern("solid", color=self.color(color), transform=transform)
        if ty in ("stripe", "gradient", "ring", "checker", "blend"):
            a = self.sub_pattern(transform, _get(p, "color_a"), _get(p, "pattern_a"))
            b = self.sub_pattern(transform, _get(p, "color_b"), _get(p, "pattern_b"))
            scale = get_f64_default(_get(p, "scale"), 0.5) if ty == "blend" else 0.5
            return self.o.pattern(ty, a=a, b=b, scale=scale, transform=transform)
        if ty == "perturbed":  # :272-281
            scale = get_f64_default(_get(p, "scale"), 0.2)
            octaves = _as_usize(get_f64_default(_get(p, "octaves"), 3.0))
            persistence = get_f64_default(_get(p, "persistence"), 0.5)
            a = self.sub_pattern(transform, _get(p, "color_a"), _get(p, "pattern_a"))
            pid = self.o.pattern("perturbed", a=a, scale=scale, transform=transform)
            self.o.set_noise(pid, octaves, persistence)
            return pid
        if ty == "noise":  # :282-292
            octaves = _as_usize(get_f64_default(_get(p, "octaves"), 1.0))
            persistence = get_f64_default(_get(p, "persistence"), 1.0)
            scale = get_f64_default(_get(p, "scale"), 1.0)
            a = self.sub_pattern(transform, _get(p, "color_a"), _get(p, "pattern_a"))
            b = self.sub_pattern(transform, _get(p, "color_b"), _get(p, "pattern_b"))
            pid = self.o.pattern("noise", a=a, b=b, scale=scale, transform=transform)
            self.o.set_noise(pid, octaves, persistence)
            return pid
        if ty == "image":  # :293-296 -> Texture::new (texture.rs:15-19): decode, to_rgba8
            path = _get(p, "file")
            if not isinstance(path, str):
                raise ValueError("file not found")
            if self.obj_root and not os.path.isabs(path):
                path = os.path.join(self.obj_root, path)
            if path not in self.textures:
                from PIL import Image

                self.textures[path] = self.o.add_texture(np.asarray(Image.open(path).convert("RGBA")))
            return self.o.pattern("texture", a=self.textures[path], transform=transform)
        return self.o.pattern("solid", color=(0.0, 0.0, 0.0), transform=transform)

    def sub_pattern(self, transform, color, pat):  # :310-317
        if isinstance(color, list):
            return self.o.pattern("solid", color=self.color(color), transform=transform)
        return self.create_pattern(pat)

    def create_material(self, m):  # :319-332 -> (mat7, pattern)
        if m is BAD:
            return DEFAULT_MAT7, -1
        mat7 = (get_f64_default(_get(m, "ambient"), 0.1), get_f64_default(_get(m, "diffuse"), 0.9),
                get_f64_default(_get(m, "specular"), 0.9), get_f64_default(_get(m, "shininess"), 200.0),
                get_f64_default(_get(m, "reflective"), 0.0), get_f64_default(_get(m, "transparency"), 0.0),
                get_f64_default(_get(m, "refractive_index"), 1.0))
        return mat7, self.create_pattern(_get(m, "pattern"))

    def create_shape(self, s, parent):  # :334-365
        ty = _get(s, "type")
        o = self.o
        if ty in ("sphere", "glass_sphere", "plane"):
            oid = o.add("plane" if ty == "plane" else "sphere", parent)
        elif ty == "triangle":
            p = [tuple(get_f64(x) for x in _get(s, k)[:3]) for k in ("p1", "p2", "p3")]
            oid = o.add_triangle(*p, parent=parent)
        elif ty == "obj_file":
            path = _get(s, "obj_file")
            if self.obj_root and not os.path.isabs(path):
                path = os.path.join(self.obj_root, path)
            mat7, pat = self.create_material(_get(s, "material"))
            oid = o.load_obj(path, parent, mat7, pat)
        elif ty == "group":
            oid = o.add("group", parent)
            for ch in _get(s, "children"):
                if _get(ch, "hidden") is not True:
                    self.create_shape(ch, oid)
        elif ty == "cube":
            oid = o.add("cube", parent)
        elif ty in ("cylinder", "cone"):  # :332-343
            oid = o.add(ty, parent)
            o.set_shape_params(oid, get_f64_default(_get(s, "minimum"), -math.inf),
                               get_f64_default(_get(s, "maximum"), math.inf), _get(s, "closed") is True)
        elif ty == "csg":  # :152-162 — left is created (and registered) before right
            op = _get(s, "operation")
            if op not in ("union", "intersection", "difference"):
                raise ValueError(f"Unknown operation: {op}")
            oid = o.add_csg(op, parent)
            self.create_shape(_get(s, "left"), oid)
            self.create_shape(_get(s, "right"), oid)
        elif ty == "torus":  # :350-353
            oid = o.add("torus", parent)
            o.set_shape_params(oid, get_f64(_get(s, "minor_radius")), math.inf, False)
        else:
            raise ValueError(f"Unknown object type: {ty}")
        ts = _get(s, "transforms")
        o.set_transform(oid, create_transforms(ts if isinstance(ts, list) else []))
        if ty not in ("group", "obj_file", "csg"):  # Group/Csg::set_material are no-ops (group.rs, csg.rs)
            # glass_sphere's material (sphere.rs:48-58) is always overwritten by create_material here
            mat7, pat = self.create_material(_get(s, "material"))
            o.set_material(oid, mat7, pat)
        else:
            self.create_material(_get(s, "material"))  # evaluated (and may panic) like the reference
        return oid


def load_yaml_text(text):
    docs = list(yaml.load_all(text.replace("\r\n", "\n").replace("\r", "\n"), Loader=_Loader))
    return docs[0]


def build_from_yaml(text, width, height, aa=1, obj_root=None):
    """render_scene_from_str (:387-410) up to camera.render: returns (Oracle, camera)."""
    doc = load_yaml_text(text)
    cam = _get(doc, "camera")
    fov = get_f64(_get(cam, "fov"))
    f = [get_f64(x) for x in _get(cam, "from")[:3]]
    t = [get_f64(x) for x in _get(cam, "to")[:3]]
    u = [get_f64(x) for x in _get(cam, "up")[:3]]
    o = Oracle()
    camera = Oracle.camera(width * aa, height * aa, deg2rad(fov), Mat.view_transform(f, t, u))
    lights = _get(doc, "lights")
    if not isinstance(lights, list) or not lights:
        raise ValueError("No lights found in scene")
    for lt in lights:  # :112-151
        ty = _get(lt, "type")
        col = [get_f64(x) for x in _get(lt, "color")[:3]]
        if ty == "point":
            o.point_light([get_f64(x) for x in _get(lt, "position")[:3]], col)
        elif ty == "area":
            lv = _get(lt, "level")
            level = lv if (isinstance(lv, int) and not isinstance(lv, bool)) else 5
            o.area_light([get_f64(x) for x in _get(lt, "corner")[:3]], [get_f64(x) for x in _get(lt, "uvec")[:3]],
                         [get_f64(x) for x in _get(lt, "vvec")[:3]], col, level)
        else:
            raise ValueError(f"Unknown light type: {ty}")
    b = YamlSceneBuilder(o, obj_root)
    for s in _get(doc, "scene"):
        if _get(s, "hidden") is not True:
            b.create_shape(s, -1)
    return o, camera

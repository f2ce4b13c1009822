"""CPU-side tests of the product library: exports, host logic (YAML front-end, flattening,
partitioning, quantisation, PNG) — no kernel launches."""
import ctypes as C
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def R():
    from rray_amd import build

    build.build()
    import rray_amd

    return rray_amd


def header_functions():
    text = open(os.path.join(ROOT, "include", "rray", "rray.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol(R):
    L = R.lib()
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    hdr = open(os.path.join(ROOT, "include", "rray", "rray.h")).read()
    assert L.rr_abi_version() == int(re.search(r"#define RR_ABI_VERSION (\d+)", hdr).group(1))
    assert sorted(R._lib.EXPORTS) == names


def test_kernel_list_matches_the_library():
    """rr_kernel_times reports K_COUNT kernels (kernels.hpp KernelId): the Python names (_lib.KERNELS) and the
    header's documented order and count must be that list.  The GPU test test_kernel_times_count_matches checks
    the call's return value."""
    from rray_amd import _lib

    kh = open(os.path.join(ROOT, "rray_amd", "csrc", "kernels.hpp")).read()
    enum = re.search(r"enum KernelId \{([^}]*)\}", kh).group(1)
    ids = [e.strip().split("=")[0].strip() for e in enum.split(",") if e.strip()]
    assert ids[-1] == "K_COUNT"
    names = [i[2:].lower() for i in ids[:-1]]
    assert names == _lib.KERNELS
    hdr = re.sub(r"\s+", " ", re.sub(r"\n\s*\*", " ", open(os.path.join(ROOT, "include", "rray", "rray.h")).read()))
    doc = re.search(r"per kernel in the order ([a-z0-9_, ]+) \(returns the number of kernels, (\d+);", hdr)
    assert doc, "rr_kernel_times documentation not found"
    assert [n.strip() for n in doc.group(1).split(",")] == _lib.KERNELS
    assert int(doc.group(2)) == len(_lib.KERNELS)


def test_no_cpu_fallback_without_device(R):
    if R.device_count() > 0:
        pytest.skip("a GPU is visible; the no-device path is exercised on CPU hosts")
    with pytest.raises(R.RRError) as e:
        R.Renderer(0)
    assert e.value.code == -2  # RR_E_HIP


def _inspect(R, desc):
    n = desc.n_objects
    inv, aabb, node = np.zeros((n, 16)), np.zeros((n, 6)), np.zeros(n, np.int32)
    R._lib.check(R.lib().rr_scene_inspect(C.byref(desc), inv.ctypes.data_as(R._lib._D),
                                          aabb.ctypes.data_as(R._lib._D), node.ctypes.data_as(R._lib._I)))
    return inv, aabb, node


YAMLS = [(SCENES, f) for f in ("c1_readme.yaml", "c2_s1024.yaml", "c3_s1024_reflect.yaml", "c4_teapot.yaml",
                               "c5_area_light.yaml")] + \
        [(GOLDEN, f) for f in ("checker_pattern.yaml", "stripe_pattern.yaml", "gradient_pattern.yaml",
                               "ring_pattern.yaml", "blend_pattern.yaml", "triangle.yaml", "objects_cylinder.yaml",
                               "objects_cone.yaml", "shapes_csg.yaml", "shapes_glass.yaml", "shapes_mixed.yaml",
                               "noise_pattern.yaml", "perturbed_pattern.yaml", "objects_sphere.yaml",
                               "objects_cube.yaml", "patterns_noise_mix.yaml", "textures_mix.yaml",
                               "shapes_torus.yaml")] + [(os.path.join(GOLDEN, "example1"), f) for f in ("example1.yaml", "torus.yaml")]


@pytest.mark.parametrize("root,name", YAMLS)
def test_yaml_front_end_matches_oracle_builder(R, oracle_mod, root, name):
    """C++ YAML parser + builder vs PyYAML + the oracle's restatement: bit-identical inverses,
    group boxes and camera (scene_builder_yaml.rs:89-365, matrix.rs:389-412, group.rs:128-149)."""
    from oracle.scene_yaml import build_from_yaml

    text = open(os.path.join(root, name)).read()
    s = R.YamlScene(text, 64, 48, 2, obj_root=root)
    o, cam = build_from_yaml(text, 64, 48, 2, obj_root=root)
    d = s.desc()
    inv, aabb, node = _inspect(R, d)
    assert o.num_objects() == d.n_objects
    for i in range(d.n_objects):
        ref = np.array(o.inverse_of(i)).reshape(4, 4)
        assert np.array_equal(inv[i].reshape(4, 4)[:3], ref[:3]), (name, i)
        if d.kind[i] in (2, 8):  # group, CSG: cached AABB (group.rs:128-149, csg.rs get_aabb)
            assert np.array_equal(aabb[i], np.array(o.group_aabb(i)), equal_nan=True), (name, i)
        if d.kind[i] in (6, 7):  # cylinder / cone parameters
            assert [d.shape[3 * i + k] for k in range(3)] == o.shape_params(i), (name, i)
        if d.kind[i] == 9:  # torus minor radius
            assert d.shape[3 * i] == o.shape_params(i)[0], (name, i)
        if d.kind[i] == 8:
            assert d.csg_op[i] == o.csg_op(i), (name, i)
    assert d.n_patterns == o.num_patterns()
    for j in range(d.n_patterns):  # pattern tree nodes in creation order (scene_builder_yaml.rs:226-317)
        kind, a, b, scale, octaves, persistence = o.pattern_info(j)
        assert (d.pat_kind[j], d.pat_a[j], d.pat_b[j]) == (kind, a, b), (name, j)
        if kind in (6, 7, 8):
            assert d.pat_scale[j] == scale, (name, j)
        if kind in (7, 8):
            assert (d.pat_octaves[j], d.pat_persistence[j]) == (octaves, persistence), (name, j)
    for f in ("hsize", "vsize", "pixel_size", "half_width", "half_height"):
        assert getattr(s.camera, f) == getattr(cam, f), f
    assert list(s.camera.transform) == list(cam.transform)


def test_yaml_edge_cases(R):
    base = "camera:\r  fov: 60\r  from: [0, 1.5, -5.0]\r  to: [0,1,0]\r  up:\r    - 0\r    - 1\r    - 0\r"
    text = base + ("lights:\r  - type: point  # comment\r    color: [.25, 1e0, 2.5E-1]\r    position: [-10,10,-10]\r"
                   "scene:\r  - type: sphere\r    transforms:\r      - type: rotate\r        axis: 'y'\r"
                   "        angle: 30\r  - type: plane\r    hidden: true\r---\rcamera: junk\r")
    s = R.YamlScene(text, 10, 10, 1)
    d = s.desc()
    assert d.n_objects == 1 and d.n_lights == 1
    assert [d.light[3 + k] for k in range(3)] == [0.25, 1.0, 0.25]
    assert math.isclose(s.camera.field_of_view, math.pi / 3)
    with pytest.raises(R.RRError):
        R.YamlScene(base + "lights: []\rscene: []\r", 10, 10, 1)  # "No lights found in scene"
    with pytest.raises(R.RRError):
        R.YamlScene(base + "lights:\r  - type: spot\r    color: [1,1,1]\rscene: []\r", 10, 10, 1)
    s = R.YamlScene(base + "lights:\r  - type: point\r    color: [1,1,1]\r    position: [0,0,0]\r"
                    "scene:\r  - type: torus\r    minor_radius: 0.25\r", 10, 10, 1)
    assert s.desc().kind[0] == R._lib.TORUS and s.desc().shape[0] == 0.25
    with pytest.raises(R.RRError) as e:  # torus.rs: minor_radius is required (get_f64 panics)
        R.YamlScene(base + "lights:\r  - type: point\r    color: [1,1,1]\r    position: [0,0,0]\r"
                    "scene:\r  - type: torus\r", 10, 10, 1)
    assert e.value.code == R._lib.RR_E_SCENE
    lights = "lights:\r  - type: point\r    color: [1,1,1]\r    position: [0,0,0]\r"
    with pytest.raises(R.RRError) as e:
        s = R.YamlScene(base + lights + "scene:\r  - type: sphere\r    material:\r      pattern:\r        type: noise\r"
                    "        octaves: 1000\r        color_a: [1, 0, 0]\r        color_b: [0, 1, 0]\r", 10, 10, 1)
        _inspect(R, s.desc())
    assert e.value.code == -5  # octaves above RR_MAX_OCTAVES


def test_obj_loader_counts(R):
    text = ("camera: {fov: 60, from: [0, 0, -5], to: [0, 0, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [0, 0, -5]\nscene:\n  - type: obj_file\n    obj_file: OBJ\n")
    s = R.YamlScene(text.replace("OBJ", "teapot-low.obj"), 8, 8, 1, obj_root=GOLDEN)
    d = s.desc()
    assert d.n_objects == 241 and d.kind[0] == 2 and d.child_count[0] == 240  # load_obj.rs:153-158
    s = R.YamlScene(text.replace("OBJ", "triangles.obj"), 8, 8, 1, obj_root=GOLDEN)
    d = s.desc()  # two all-triangle models: tobj leaves face_arities empty -> empty groups
    assert d.n_objects == 3 and all(d.child_count[i] == 0 for i in (1, 2))


def test_partition_rows(R):
    for H in (1, 7, 1080, 2160):
        for n in (1, 2, 3, 4, 8):
            allrows = np.concatenate([R.part_rows(H, p, n, 8) for p in range(n)])
            assert np.array_equal(np.sort(allrows), np.arange(H)), (H, n)


def test_quantize_and_png(R, oracle_mod, tmp_path):
    rng = np.random.default_rng(0)
    avg = rng.uniform(-0.2, 1.3, (5, 7, 3))
    avg[0, 0] = [np.nan, np.inf, -np.inf]
    q = R.quantize(avg)
    assert np.array_equal(q, oracle_mod.Oracle.quantize(avg))
    assert list(q[0, 0]) == [0, 255, 0, 255]
    p = str(tmp_path / "x.png")
    R.write_png(p, q)
    from PIL import Image

    assert np.array_equal(np.array(Image.open(p).convert("RGBA")), q)


def test_camera_new_matches_oracle(R, oracle_mod):
    M = oracle_mod.Oracle.mat
    t = M.view_transform((0, 1.5, -5), (0, 1, 0), (0, 1, 0))
    for hs, vs in ((160, 120), (125, 200), (1920, 1080)):
        a = R.camera(hs, vs, math.pi / 3, t)
        b = oracle_mod.Oracle.camera(hs, vs, math.pi / 3, t)
        assert (a.pixel_size, a.half_width, a.half_height) == (b.pixel_size, b.half_width, b.half_height)


def test_jitter_is_deterministic_and_uniform(oracle_mod):
    v = np.array([oracle_mod.Oracle.jitter(0, s, 1, 0, k, 0) for s in range(200) for k in range(25)])
    assert v.min() >= 0 and v.max() < 1 and abs(v.mean() - 0.5) < 0.02


def test_shape_and_csg_descriptor_checks(R):
    """A CSG needs a left and a right child (csg.rs panics on get_object(usize::MAX)); CSG subtrees
    are bounded by RR_MAX_CSG_ENTRIES intersections per ray."""
    b = R.SceneBuilder()
    b.point_light((-10, 10, -10), (1, 1, 1))
    c = b.csg("union")
    b.sphere(parent=c)
    with pytest.raises(R.RRError) as e:
        _inspect(R, b.desc())
    assert e.value.code == R._lib.RR_E_SCENE
    b = R.SceneBuilder()
    b.point_light((-10, 10, -10), (1, 1, 1))
    c = b.csg("union")
    g = b.group(parent=c)
    for _ in range(9):
        b.cylinder(-1, 1, True, parent=g)
    b.sphere(parent=c)
    with pytest.raises(R.RRError) as e:
        _inspect(R, b.desc())
    assert e.value.code == R._lib.RR_E_LIMIT


def test_png_texture_decoder_matches_pil(R):
    """The product front-end's PNG reader (texture.rs:15-19: decode, to_rgba8) against PIL on RGB,
    4-bit palette, grey and RGBA files: the colour channels the sampler reads must be identical."""
    from PIL import Image

    files = ["tex_grid.png", "tex_pal.png", "tex_grey.png", "test_texture.png", "triangle.png"]
    scene = "".join(f"  - type: sphere\n    material: {{pattern: {{type: image, file: 'png/{f}'}}}}\n" for f in files)
    text = ("camera: {fov: 60, from: [0, 0, -5], to: [0, 0, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [0, 0, -5]\nscene:\n" + scene)
    s = R.YamlScene(text, 8, 8, 1, obj_root=GOLDEN)
    d = s.desc()
    assert d.n_textures == len(files)
    off = 0
    for i, f in enumerate(files):
        w, h = d.tex_size[2 * i], d.tex_size[2 * i + 1]
        got = np.ctypeslib.as_array(d.texels, shape=(off + w * h * 4,))[off:].reshape(h, w, 4)
        ref = np.asarray(Image.open(os.path.join(GOLDEN, "png", f)).convert("RGBA"))
        assert got.shape == ref.shape, f
        assert np.array_equal(got[..., :3], ref[..., :3]), f
        off += w * h * 4
    # the same file twice is decoded once (both patterns share the texture)
    s2 = R.YamlScene(text.replace("tex_pal", "tex_grid"), 8, 8, 1, obj_root=GOLDEN)
    assert s2.desc().n_textures == len(files) - 1
    with pytest.raises(R.RRError) as e:
        R.YamlScene(text.replace("tex_grid.png", "missing.png"), 8, 8, 1, obj_root=GOLDEN)
    assert e.value.code == R._lib.RR_E_IO
    with pytest.raises(R.RRError) as e:  # JPEG (examples/Texturelabs_Stone_138M.jpg): host-side decode only
        R.YamlScene(text.replace("png/tex_grid.png", "teapot-low.obj"), 8, 8, 1, obj_root=GOLDEN)
    assert e.value.code == R._lib.RR_E_LIMIT


def test_png_interlaced_and_16bit_textures(R, tmp_path):
    """Adam7-interlaced PNGs (every colour type and bit depth the image crate decodes) equal PIL's decoding; 16-bit
    samples become 8 bits as image's to_rgba8 converts them, round(c * 255 / 65535) = (c + 128) / 257 (image 0.25
    FromPrimitive<u16> for u8; parity unpinned: no reference-held 16-bit PNG, and PIL truncates instead)."""
    from PIL import Image

    from png_helpers import png_bytes

    rng = np.random.default_rng(11)
    cases = []
    for ctype, depth, ch in ((2, 8, 3), (6, 8, 4), (0, 8, 1), (4, 8, 2), (0, 4, 1), (0, 1, 1), (3, 2, 1), (3, 8, 1),
                             (2, 16, 3), (6, 16, 4), (0, 16, 1), (4, 16, 2)):
        for interlace in (0, 1):
            h, w = int(rng.integers(1, 23)), int(rng.integers(1, 23))
            hi = (1 << depth) - 1 if ctype != 3 else (1 << depth) - 1
            img = rng.integers(0, hi + 1, size=(h, w, ch)).astype(np.uint16 if depth == 16 else np.uint8)
            pal = rng.integers(0, 256, size=3 * (1 << depth)).tolist() if ctype == 3 else None
            name = f"t_{ctype}_{depth}_{interlace}.png"
            (tmp_path / name).write_bytes(png_bytes(img, ctype, depth, interlace, pal))
            cases.append((name, ctype, depth, img, pal))
    scene = "".join(f"  - type: sphere\n    material: {{pattern: {{type: image, file: '{c[0]}'}}}}\n" for c in cases)
    text = ("camera: {fov: 60, from: [0, 0, -5], to: [0, 0, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [0, 0, -5]\nscene:\n" + scene)
    scn = R.YamlScene(text, 8, 8, 1, obj_root=str(tmp_path))  # owns the descriptor's arrays
    d = scn.desc()
    assert d.n_textures == len(cases)
    off = 0
    for i, (name, ctype, depth, img, pal) in enumerate(cases):
        w, h = d.tex_size[2 * i], d.tex_size[2 * i + 1]
        got = np.ctypeslib.as_array(d.texels, shape=(off + w * h * 4,))[off:].reshape(h, w, 4)[..., :3]
        off += w * h * 4
        assert (h, w) == img.shape[:2], name
        if depth == 16:
            want8 = ((img.astype(np.uint32) + 128) // 257).astype(np.uint8)
            want = np.repeat(want8[..., :1], 3, axis=2) if ctype in (0, 4) else want8[..., :3]
            if ctype == 0:  # PIL keeps 16-bit grey ("I;16"): the same conversion applied to PIL's samples
                ref16 = np.asarray(Image.open(tmp_path / name), dtype=np.uint32)
                assert np.array_equal(((ref16 + 128) // 257).astype(np.uint8), want8[..., 0]), name
        else:
            want = np.asarray(Image.open(tmp_path / name).convert("RGB"))
        assert np.array_equal(got, want), name


def test_other_texture_formats_match_pil(R, tmp_path):
    """BMP (1 / 4 / 8-bit palette, 24-bit, 32-bit bitfields, top-down), TGA (grey, RGB, RGBA, colour-mapped, raw and
    run-length, both origins), PNM (P1-P6) and GIF (plain and interlaced) — the formats image::open decodes with its
    default features (texture.rs:15-19) — decoded by the product front-end equal PIL's decoding of the same files."""
    from PIL import Image

    rng = np.random.default_rng(5)

    def rgb(h, w):
        return Image.fromarray(rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8), "RGB")

    files = []

    def add(name, img, **kw):
        img.save(tmp_path / name, **kw)
        files.append(name)

    add("a.bmp", rgb(13, 17))
    add("b.bmp", rgb(9, 6).convert("P", palette=Image.ADAPTIVE, colors=200))
    add("c.bmp", rgb(7, 11).convert("1"))
    add("d.bmp", rgb(5, 9).convert("L"))
    add("e.bmp", Image.fromarray(rng.integers(0, 256, size=(6, 7, 4), dtype=np.uint8), "RGBA"))
    add("f.tga", rgb(10, 12))
    add("g.tga", rgb(10, 12), compression="tga_rle")
    add("h.tga", Image.fromarray(rng.integers(0, 256, size=(5, 8, 4), dtype=np.uint8), "RGBA"), compression="tga_rle")
    add("i.tga", rgb(7, 5).convert("L"))
    add("j.tga", rgb(7, 5).convert("P", palette=Image.ADAPTIVE, colors=64))
    add("k.tga", rgb(6, 9), orientation=1)
    add("l.ppm", rgb(8, 11))
    add("m.pgm", rgb(8, 11).convert("L"))
    add("n.pbm", rgb(9, 13).convert("1"))
    add("o.gif", rgb(12, 14))
    add("p.gif", rgb(19, 23), interlace=True)
    add("q.gif", Image.fromarray(np.tile(np.arange(250, dtype=np.uint8), (40, 1)), "L"))
    # the ASCII PNM variants (PIL writes binary ones) and a 4-bit palette BMP, by hand
    a = rng.integers(0, 256, size=(3, 4, 3))
    (tmp_path / "r.ppm").write_text("P3\n# comment\n4 3\n255\n" + " ".join(str(int(v)) for v in a.reshape(-1)) + "\n")
    g = rng.integers(0, 256, size=(3, 5))
    (tmp_path / "s.pgm").write_text("P2 5 3 255\n" + "\n".join(" ".join(str(int(v)) for v in r) for r in g) + "\n")
    b = rng.integers(0, 2, size=(2, 9))
    (tmp_path / "t.pbm").write_text("P1\n9 2\n" + "\n".join("".join(str(int(v)) for v in r) for r in b) + "\n")
    files += ["r.ppm", "s.pgm", "t.pbm"]
    scene = "".join(f"  - type: sphere\n    material: {{pattern: {{type: image, file: '{f}'}}}}\n" for f in files)
    text = ("camera: {fov: 60, from: [0, 0, -5], to: [0, 0, 0], up: [0, 1, 0]}\nlights:\n  - type: point\n"
            "    color: [1, 1, 1]\n    position: [0, 0, -5]\nscene:\n" + scene)
    scn = R.YamlScene(text, 8, 8, 1, obj_root=str(tmp_path))
    d = scn.desc()
    assert d.n_textures == len(files)
    off = 0
    for i, f in enumerate(files):
        w, h = d.tex_size[2 * i], d.tex_size[2 * i + 1]
        got = np.ctypeslib.as_array(d.texels, shape=(off + w * h * 4,))[off:].reshape(h, w, 4)[..., :3]
        off += w * h * 4
        ref = np.asarray(Image.open(tmp_path / f).convert("RGB"))
        assert got.shape == ref.shape, f
        assert np.array_equal(got, ref), f
    with pytest.raises(R.RRError) as e:  # an unknown format is refused, not misread
        (tmp_path / "u.xyz").write_bytes(b"\x00\x01garbage")
        R.YamlScene(text.replace("'a.bmp'", "'u.xyz'"), 8, 8, 1, obj_root=str(tmp_path))
    assert e.value.code == R._lib.RR_E_LIMIT


def test_corrupt_textures_under_asan(tmp_path):
    """The texture reader (png.cpp, jpeg.cpp, imgfmt.cpp: host code) built with g++ -fsanitize=address, on files of
    every format truncated at random points and with random bytes flipped: each is decoded or refused with an error
    code, with no out-of-bounds access reported (and a decoded image always holds width x height texels)."""
    import shutil
    import subprocess

    from PIL import Image

    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path / "img_asan")
    csrc = os.path.join(ROOT, "rray_amd", "csrc")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                        "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "asan_image_main.cpp"),
                        os.path.join(csrc, "png.cpp"), os.path.join(csrc, "jpeg.cpp"), os.path.join(csrc, "imgfmt.cpp"),
                        "-lz", "-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("AddressSanitizer unavailable")
    assert r.returncode == 0, r.stderr
    rng = np.random.default_rng(17)
    img = Image.fromarray(rng.integers(0, 256, size=(13, 11, 3), dtype=np.uint8), "RGB")
    seeds = []
    for name, kw in (("s.png", {}), ("s.jpg", {"quality": 80}), ("s.bmp", {}), ("s.tga", {"compression": "tga_rle"}),
                     ("s.ppm", {}), ("s.gif", {"interlace": True})):
        img.save(tmp_path / name, **kw)
        seeds.append(tmp_path / name)
    img.convert("P", palette=Image.ADAPTIVE, colors=16).save(tmp_path / "p.bmp")
    seeds.append(tmp_path / "p.bmp")
    files = []
    for sd in seeds:
        data = bytearray(sd.read_bytes())
        for k in range(24):
            m = bytearray(data)
            if k % 3 == 0:
                m = m[: int(rng.integers(1, len(m)))]
            else:
                for _ in range(1 + k % 5):
                    m[int(rng.integers(0, len(m)))] = int(rng.integers(0, 256))
            f = tmp_path / f"{sd.stem}_{k}{sd.suffix}"
            f.write_bytes(bytes(m))
            files.append(str(f))
    # GIF frames larger than the texel limit or empty: refused from the image descriptor, before the LZW buffers
    # are sized (a 30-byte file must not reach a multi-GB allocation)
    gif = bytearray((tmp_path / "s.gif").read_bytes())
    at = gif.index(b"\x2c\x00\x00\x00\x00")  # the image descriptor (frame at 0, 0)
    bad = []
    for fw, fh in ((65535, 65535), (0, 13), (11, 0)):
        m = bytearray(gif)
        m[at + 5:at + 9] = bytes([fw & 255, fw >> 8, fh & 255, fh >> 8])
        f = tmp_path / f"frame_{fw}x{fh}.gif"
        f.write_bytes(bytes(m))
        bad.append(str(f))
    files += bad
    r = subprocess.run([exe] + [str(s) for s in seeds] + files, capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0, r.stderr[-3000:]
    rcs = [int(line.split()[0]) for line in r.stdout.splitlines()]
    assert len(rcs) == len(seeds) + len(files)
    assert rcs[: len(seeds)] == [0] * len(seeds)  # the intact files decode
    assert all(rc != 0 for rc in rcs[-len(bad):])  # the oversized and empty GIF frames are refused


def test_group_contexts_need_a_device(R):
    """rr_create_multi / rr_create_rank validate their arguments and, like rr_create, have no CPU
    fallback (the multi-GPU path itself runs in tests/test_gpu_multi.py)."""
    with pytest.raises(R.RRError) as e:
        R.Renderer.multi([])
    assert e.value.code == -1  # RR_E_ARG
    with pytest.raises(R.RRError) as e:
        R.Renderer.rank(0, 2, 5, bytes(R._lib.RCCL_ID_BYTES))
    assert e.value.code == -1
    if R.device_count() == 0:
        with pytest.raises(R.RRError) as e:
            R.Renderer.multi([0])
        assert e.value.code == -2  # RR_E_HIP


def test_cli_argument_errors():
    """The drop-in CLI's clap-style errors (main.rs:13-45) and the missing-file panic
    (scene_builder_yaml.rs:434) as an exit code — none of these touch the GPU."""
    import subprocess

    cli = os.path.join(ROOT, "rray_amd", "bin", "rray")
    r = subprocess.run([cli, "-W", "10"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "--scene <SCENE>" in r.stderr
    r = subprocess.run([cli, "-s", "x.yaml", "-a", "6"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "less than or equal to 5" in r.stderr
    r = subprocess.run([cli, "-s", "x.yaml", "-W", "-3"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    r = subprocess.run([cli, "-s", os.path.join(ROOT, "no_such_scene.yaml")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1 and "File does not exist" in r.stderr
    r = subprocess.run([cli, "-V"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.startswith("rray")


def test_balance_bands():
    """rr_balance_bands (ABI 10, partition.hpp balance_bands): the multi-device bands from per-row costs — bounds from 0
    to height, non-decreasing, inner bounds on `align` rows; equal costs give equal bands; a costly region gets thinner
    bands; rank 0's extra (its transfer work) shrinks band 0 by about that much cost; degenerate inputs stay valid."""
    import rray_amd as R

    b = R.balance_bands(np.ones(2160), 8)  # the even split 270 p, on 8-row boundaries
    assert b[0] == 0 and b[-1] == 2160 and all(x % 8 == 0 and abs(x - 270 * p) <= 4 for p, x in enumerate(b[:-1]))
    cost = np.ones(800)
    cost[400:] = 3.0  # the lower half three times as costly
    b = R.balance_bands(cost, 4)
    assert b[0] == 0 and b[-1] == 800 and all(x % 8 == 0 for x in b[:-1])
    sums = [cost[b[p]:b[p + 1]].sum() for p in range(4)]
    assert max(sums) - min(sums) <= 8 * 3.0  # within one aligned block of the most costly rows
    b0 = R.balance_bands(np.ones(2160), 8, root_extra=80.0)
    assert 0 < b0[1] < 270 and abs((b0[1] + 80.0) - (2160 + 80.0) / 8) <= 8
    big = R.balance_bands(np.ones(64), 4, root_extra=1e6)  # the root's extra outweighs the frame: rank 0 gets no rows
    assert big[0] == big[1] == 0 and big[-1] == 64
    z = R.balance_bands(np.zeros(100), 3)  # no cost information: still a valid partition
    assert z[0] == 0 and z[-1] == 100 and all(x <= y for x, y in zip(z, z[1:]))
    many = R.balance_bands(np.ones(16), 8)  # more parts than 8-row blocks: some bands empty
    assert many[0] == 0 and many[-1] == 16 and all(x <= y for x, y in zip(many, many[1:]))
    nan = np.ones(64)
    nan[10] = np.nan
    assert R.balance_bands(nan, 2)[-1] == 64
    with pytest.raises(R.RRError):
        R.balance_bands(np.ones(10), 0)

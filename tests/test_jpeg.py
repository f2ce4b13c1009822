"""JPEG textures (texture.rs:15-19: Texture::new decodes any image file, then to_rgba8) through the
product front-end's decoder (rray_amd/csrc/jpeg.cpp), CPU only.

The reference decodes with the image crate 0.25 (zune-jpeg, not vendored and not importable here);
the oracle decodes textures with PIL (libjpeg-turbo).  The product decoder restates libjpeg's
integer islow IDCT, YCbCr tables and fancy upsampling, so its texels must equal PIL's bit for bit —
on the reference's own texture (examples/Texturelabs_Stone_138M.jpg, used by
examples/objects/torus.yaml) and on synthetic files PIL writes here: 4:4:4 / 4:2:2 / 4:2:0 / grey,
baseline and progressive (spectral selection + successive approximation), restart intervals,
optimised Huffman tables, odd and tiny sizes.  Parity with zune-jpeg itself is unpinned (no
reference-held output decodes this file: torus.png predates its scene).
"""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX1 = os.path.join(ROOT, "tests", "golden", "example1")
REF_JPEG = os.path.join(EX1, "examples", "Texturelabs_Stone_138M.jpg")

PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module")
def R():
    from rray_amd import build

    build.build()
    import rray_amd

    return rray_amd


SCENE = """camera:
  fov: 60
  from: [0, 0, -5]
  to: [0, 0, 0]
  up: [0, 1, 0]
lights:
  - type: point
    position: [-10, 10, -10]
    color: [1, 1, 1]
scene:
  - type: sphere
    transforms: []
    material:
      pattern:
        type: image
        file: '{path}'
        transforms: []
"""


def texels(R, path):
    """The decoded RGBA8 texels the front-end hands to the device (rr_scene_desc.texels)."""
    s = R.YamlScene(SCENE.format(path=path), 8, 8, 1)
    d = s.desc()
    assert d.n_textures == 1
    w, h = d.tex_size[0], d.tex_size[1]
    return np.ctypeslib.as_array(d.texels, (h, w, 4)).copy()


def pil_rgba(path):
    return np.asarray(PIL.open(path).convert("RGBA"))


def smooth(h, w):
    yy, xx = np.mgrid[0:h, 0:w]
    return np.stack([128 + 100 * np.sin(xx / 7 + yy / 11), 128 + 90 * np.cos(xx / 5 - yy / 9),
                     128 + 60 * np.sin(xx * yy / 300)], -1).astype(np.uint8)


def noise(h, w, seed=1):
    return (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)


def test_reference_texture_matches_pil(R):
    """The reference's own JPEG (1920x1281, baseline, 4:4:4, Adobe APP14 YCbCr): every texel."""
    got, ref = texels(R, REF_JPEG), pil_rgba(REF_JPEG)
    assert got.shape == ref.shape == (1281, 1920, 4)
    assert np.array_equal(got, ref), int((got != ref).any(axis=2).sum())


@pytest.mark.parametrize("progressive", [False, True])
@pytest.mark.parametrize("subsampling", [0, 1, 2])  # 4:4:4, 4:2:2, 4:2:0
@pytest.mark.parametrize("quality", [30, 95, 100])
@pytest.mark.parametrize("image", ["smooth", "noise"])
def test_synthetic_jpeg_matches_pil(R, tmp_path, progressive, subsampling, quality, image):
    a = smooth(101, 77) if image == "smooth" else noise(45, 61)
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(a).save(p, quality=quality, subsampling=subsampling, progressive=progressive)
    got, ref = texels(R, p), pil_rgba(p)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), int((got != ref).any(axis=2).sum())


@pytest.mark.parametrize("kw", [dict(restart_marker_blocks=3), dict(restart_marker_blocks=2, progressive=True),
                                dict(optimize=True, subsampling=2), dict(optimize=True, progressive=True),
                                dict(restart_marker_rows=1, subsampling=1)])
def test_jpeg_options_match_pil(R, tmp_path, kw):
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(smooth(70, 93)).save(p, quality=80, **kw)
    assert np.array_equal(texels(R, p), pil_rgba(p))


@pytest.mark.parametrize("shape", [(1, 1), (1, 17), (17, 1), (3, 3), (4, 5), (5, 4), (8, 8), (9, 15), (16, 33)])
@pytest.mark.parametrize("subsampling", [0, 1, 2])
def test_jpeg_small_and_odd_sizes(R, tmp_path, shape, subsampling):
    """Partial MCUs, chroma rows of 1-2 samples (replicated, not triangle-filtered: jdsample.c) and
    single chroma rows / columns (the upsampler's edge cases)."""
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(noise(*shape, seed=shape[0] * 100 + shape[1])).save(p, quality=90, subsampling=subsampling)
    assert np.array_equal(texels(R, p), pil_rgba(p))


@pytest.mark.parametrize("progressive", [False, True])
def test_grey_jpeg(R, tmp_path, progressive):
    p = str(tmp_path / "g.jpg")
    PIL.fromarray(smooth(51, 39)[:, :, 1]).save(p, quality=85, progressive=progressive)
    assert np.array_equal(texels(R, p), pil_rgba(p))


def test_jpeg_outside_the_decoder_is_refused(R, tmp_path):
    """CMYK (4 components) -> RR_E_LIMIT; a truncated header -> RR_E_IO.  The reference would decode
    CMYK through the image crate; texels from such a file go through rr_scene_desc.texels."""
    p = str(tmp_path / "cmyk.jpg")
    PIL.fromarray(smooth(16, 16)).convert("CMYK").save(p, quality=90)
    with pytest.raises(R.RRError) as e:
        texels(R, p)
    assert e.value.code == -5
    q = tmp_path / "cut.jpg"
    q.write_bytes(open(REF_JPEG, "rb").read()[:200])
    with pytest.raises(R.RRError) as e:
        texels(R, str(q))
    assert e.value.code == -6


def _with_segment_before_sos(data: bytes, seg: bytes) -> bytes:
    at = data.index(b"\xff\xda")
    return data[:at] + seg + data[at:]


@pytest.mark.parametrize("counts", [[3] + [0] * 15, [2, 3] + [0] * 14, [0] * 6 + [127, 3] + [0] * 8])
def test_oversubscribed_huffman_table_is_refused(R, tmp_path, counts):
    """A DHT whose codes do not fit their lengths (T.81 C.2: an l-bit code must stay below 2^l) is a
    corrupt file (RR_E_IO), refused before its lookahead-table write (each of these would index the 9-bit
    lookahead at 512 or beyond: an extra 1-bit, 2-bit or 8-bit code)."""
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(smooth(16, 16)).save(p, quality=90)
    body = bytes([0x00]) + bytes(counts) + bytes(range(sum(counts)))
    seg = b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body
    q = tmp_path / "bad.jpg"
    q.write_bytes(_with_segment_before_sos(open(p, "rb").read(), seg))
    with pytest.raises(R.RRError) as e:
        texels(R, str(q))
    assert e.value.code == -6


def test_empty_scan_header_is_refused(R, tmp_path):
    """An SOS segment of length 2 (no component count) at the end of the file: RR_E_IO, no read past it."""
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(smooth(16, 16)).save(p, quality=90)
    data = open(p, "rb").read()
    q = tmp_path / "sos.jpg"
    q.write_bytes(data[:data.index(b"\xff\xda")] + b"\xff\xda\x00\x02")
    with pytest.raises(R.RRError) as e:
        texels(R, str(q))
    assert e.value.code == -6


def test_corrupt_jpegs_under_asan(tmp_path):
    """The decoder itself (jpeg.cpp, host code) built with g++ -fsanitize=address on the corrupt files
    above: every one is refused (RR_E_IO) with no out-of-bounds access reported."""
    import shutil
    import subprocess

    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path / "jpeg_asan")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                        "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "asan_jpeg_main.cpp"),
                        os.path.join(ROOT, "rray_amd", "csrc", "jpeg.cpp"), "-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("AddressSanitizer unavailable")
    assert r.returncode == 0, r.stderr
    p = str(tmp_path / "t.jpg")
    PIL.fromarray(smooth(16, 16)).save(p, quality=90)
    data = open(p, "rb").read()
    files = []
    for i, counts in enumerate([[3] + [0] * 15, [2, 3] + [0] * 14, [0] * 6 + [127, 3] + [0] * 8]):
        body = bytes([0x00]) + bytes(counts) + bytes(range(sum(counts)))
        f = tmp_path / f"dht{i}.jpg"
        f.write_bytes(_with_segment_before_sos(data, b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body))
        files.append(str(f))
    f = tmp_path / "sos.jpg"
    f.write_bytes(data[:data.index(b"\xff\xda")] + b"\xff\xda\x00\x02")
    files.append(str(f))
    r = subprocess.run([exe, p] + files, capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0, r.stderr[-3000:]
    rcs = [int(line.split()[0]) for line in r.stdout.splitlines()]
    assert rcs == [0] + [-6] * len(files), r.stdout

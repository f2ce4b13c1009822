"""The oracle against the reference renderer's own output: the PNGs that ship with the reference
(examples/patterns/*.png, examples/objects/*.png; copied to tests/golden/png with their YAML) were
rendered by the Rust binary at 800x400.  The oracle renders the same YAML, box-averages and
quantises (`as u8`, canvas.rs:76-105), and must reproduce every pixel.  The pattern scenes were
rendered with aa=1, the objects scenes with aa=3 (every other aa leaves ~7 % of the edge pixels
different; aa=3 leaves none).  noise_pattern / perturbed_pattern and objects/sphere, objects/cube
(blends of noise patterns) pin the fastnoise-lite 1.1.1 Perlin restatement (oracle/rray_oracle.cpp,
namespace fnl) and noise.rs:octave_perlin.  example1.png (the README's headline image: torus through
roots 0.0.8's quartic solver, the earthmap texture, noise, perturbed, CSG, cube / cylinder / cone,
the full teapot OBJ, reflection and refraction) pins everything at once at aa=3."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

CASES = [("checker_pattern.yaml", "checker_pattern.png", 1), ("stripe_pattern.yaml", "stripe_pattern.png", 1),
         ("ring_pattern.yaml", "ring_pattern.png", 1), ("gradient_pattern.yaml", "gradient_pattern.png", 1),
         ("blend_pattern.yaml", "blend_pattern.png", 1), ("triangle.yaml", "triangle.png", 3),
         ("objects_cylinder.yaml", "objects_cylinder.png", 3), ("objects_cone.yaml", "objects_cone.png", 3),
         ("noise_pattern.yaml", "noise_pattern.png", 1), ("perturbed_pattern.yaml", "perturbed_pattern.png", 1),
         ("objects_sphere.yaml", "objects_sphere.png", 3), ("objects_cube.yaml", "objects_cube.png", 3)]


def _png_rgb(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGB"))


@pytest.mark.parametrize("scene,png,aa", CASES)
def test_oracle_reproduces_reference_png(oracle_mod, scene, png, aa):
    pytest.importorskip("PIL")
    from oracle.scene_yaml import build_from_yaml

    text = open(os.path.join(GOLDEN, scene)).read()
    o, cam = build_from_yaml(text, 800, 400, aa, obj_root=GOLDEN)
    canvas, _ = o.render(cam, max_depth=5, threads=min(8, os.cpu_count() or 1))
    q = o.quantize(o.aa_average(canvas, aa))[..., :3]
    ref = _png_rgb(os.path.join(GOLDEN, "png", png))
    assert q.shape == ref.shape
    diff = int((q != ref).any(axis=2).sum())
    assert diff == 0, f"{diff} pixels differ from the reference's {png}"


def test_oracle_reproduces_readme_test1(oracle_mod):
    """C1's own golden: examples/test1.png is the README scene (README.md:56-113, committed as
    scenes/c1_readme.yaml) rendered by `rray -W 800 -H 400` at the CLI's default aa=1 (main.rs:49-71).
    The only reference-held image of the glass sphere (reflective 0.9, transparency 0.1): reflect,
    refract, Schlick and the n1/n2 container walk together."""
    pytest.importorskip("PIL")
    from oracle.scene_yaml import build_from_yaml

    text = open(os.path.join(ROOT, "scenes", "c1_readme.yaml")).read()
    o, cam = build_from_yaml(text, 800, 400, 1, obj_root=os.path.join(ROOT, "scenes"))
    canvas, st = o.render(cam, max_depth=5, threads=min(8, os.cpu_count() or 1))
    assert st["shade_events"] > 0
    q = o.quantize(o.aa_average(canvas, 1))[..., :3]
    ref = _png_rgb(os.path.join(GOLDEN, "png", "test1.png"))
    diff = int((q != ref).any(axis=2).sum())
    assert diff == 0, f"{diff} pixels differ from the reference's test1.png"


def test_oracle_reproduces_example1(oracle_mod):
    """/root/reference/example1.png (800x400, aa=3) from example1.yaml with its examples/ files."""
    pytest.importorskip("PIL")
    from oracle.scene_yaml import build_from_yaml

    root = os.path.join(GOLDEN, "example1")
    text = open(os.path.join(root, "example1.yaml")).read()
    o, cam = build_from_yaml(text, 800, 400, 3, obj_root=root)
    canvas, st = o.render(cam, max_depth=5, threads=min(8, os.cpu_count() or 1))
    assert st["torus_tests"] > 0
    q = o.quantize(o.aa_average(canvas, 3))[..., :3]
    ref = _png_rgb(os.path.join(root, "example1.png"))
    diff = int((q != ref).any(axis=2).sum())
    assert diff == 0, f"{diff} pixels differ from the reference's example1.png"


def test_committed_golden_renders_match_live_oracle(oracle_mod):
    """tests/golden/oracle_*.npy (the GPU suite's committed vectors, make_golden.py) are what the pinned
    oracle renders today, including each BASELINE config at its own AA (C3 aa=3, C4 aa=2)."""
    import json

    from oracle.scene_yaml import build_from_yaml

    meta = json.load(open(os.path.join(GOLDEN, "golden_renders.json")))
    assert {(g["scene"], g["aa"]) for g in meta} >= {("c3_s1024_reflect.yaml", 3), ("c4_teapot.yaml", 2)}
    for g in meta:
        text = open(os.path.join(ROOT, "scenes", g["scene"])).read()
        o, cam = build_from_yaml(text, g["W"], g["H"], g["aa"], obj_root=os.path.join(ROOT, "scenes"))
        canvas, st = o.render(cam, max_depth=5, seed=g["seed"], threads=min(8, os.cpu_count() or 1))
        assert np.array_equal(o.aa_average(canvas, g["aa"]), np.load(os.path.join(GOLDEN, g["file"]))), g["file"]
        assert st["rays"] == g["stats"]["rays"] and st["shade_events"] == g["stats"]["shade_events"], g["file"]

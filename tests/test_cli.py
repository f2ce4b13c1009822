"""The drop-in CLI `rray_amd/bin/rray` (src/main.rs:49-77): YAML file -> GPU -> PNG file on disk.

CPU tests cover argument handling (clap's defaults and refusals, main.rs:21-27), which never reaches
the GPU.  The GPU tests run the binary end to end and compare the PNG it wrote with the reference's
own output (README example1.png; examples/objects/cube.png) — the scene's relative asset paths
(`examples/teapot.obj`, `examples/earthmap.png`) resolve against the working directory, as they do
for the Rust binary (scene_builder_yaml.rs:429-436).
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "rray_amd", "bin", "rray")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _run(args, cwd=None, env=None, timeout=120):
    if not os.path.exists(CLI):
        pytest.fail("rray_amd/bin/rray is not built (run __graft_entry__.build())")
    return subprocess.run([CLI] + args, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


def test_cli_help_and_version():
    r = _run(["--help"])
    assert r.returncode == 0
    assert "Usage: rray [OPTIONS] --scene <SCENE>" in r.stderr
    for flag in ("--width", "--height", "--scene", "--output", "--aa"):
        assert flag in r.stderr
    r = _run(["-V"])
    assert r.returncode == 0 and r.stdout.startswith("rray ")


@pytest.mark.parametrize("args,msg", [
    ([], "--scene <SCENE>"),                                      # scene is required
    (["-s", "x.yaml", "-a", "6"], "less than or equal to 5"),     # main.rs:21-27 (max 5)
    (["-s", "x.yaml", "-a", "-1"], "positive number"),
    (["-s", "x.yaml", "-W", "abc"], "positive number"),
    (["-s", "x.yaml", "--bogus"], "unexpected argument"),
    (["-s"], "missing value"),
])
def test_cli_refuses_bad_arguments(args, msg):
    r = _run(args)
    assert r.returncode == 2, (r.returncode, r.stderr)
    assert msg in r.stderr


def _png(path):
    PIL = pytest.importorskip("PIL.Image")
    return np.asarray(PIL.open(path).convert("RGB"))


@pytest.mark.gpu
def test_cli_renders_example1_png(tmp_path):
    """`rray -W 800 -H 400 -s example1.yaml -o out.png -a 3` from the scene's directory writes the
    README image pixel for pixel (torus, texture, noise, CSG, teapot, reflection, refraction)."""
    out = tmp_path / "example1_cli.png"
    r = _run(["-W", "800", "-H", "400", "-s", "example1.yaml", "-o", str(out), "-a", "3"],
             cwd=os.path.join(GOLDEN, "example1"))
    assert r.returncode == 0, r.stderr
    got = _png(out)
    ref = _png(os.path.join(GOLDEN, "example1", "example1.png"))
    assert got.shape == ref.shape == (400, 800, 3)
    diff = int((got != ref).any(axis=2).sum())
    print(f"CLI example1.png: {diff} of {ref.shape[0] * ref.shape[1]} pixels differ")
    assert diff == 0


@pytest.mark.gpu
def test_cli_defaults_and_devices_env(tmp_path):
    """Default output name `output.png` in the working directory (main.rs:60-61), the default
    800x600 size, and RRAY_DEVICES=0 (the multi-device path with one device) giving the same file."""
    scene = os.path.join(GOLDEN, "objects_cube.yaml")
    r = _run(["-s", scene], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    a = _png(tmp_path / "output.png")
    assert a.shape == (600, 800, 3)
    env = dict(os.environ, RRAY_DEVICES="0")
    r = _run(["-s", scene, "-o", str(tmp_path / "multi.png")], env=env)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(a, _png(tmp_path / "multi.png"))


@pytest.mark.gpu
def test_cli_reference_cube_png(tmp_path):
    """examples/objects/cube.png (800x400, aa=3) written by the CLI, compared after decode."""
    out = tmp_path / "cube.png"
    r = _run(["-W", "800", "-H", "400", "-s", os.path.join(GOLDEN, "objects_cube.yaml"), "-o", str(out),
              "-a", "3"])
    assert r.returncode == 0, r.stderr
    ref = _png(os.path.join(GOLDEN, "png", "objects_cube.png"))
    assert int((_png(out) != ref).any(axis=2).sum()) == 0


@pytest.mark.gpu
def test_cli_missing_scene_file_fails(tmp_path):
    r = _run(["-s", str(tmp_path / "nope.yaml"), "-o", str(tmp_path / "o.png")])
    assert r.returncode == 1
    assert "rray:" in r.stderr
    assert not (tmp_path / "o.png").exists()


@pytest.mark.gpu
def test_cli_renders_torus_jpeg_scene(tmp_path):
    """`rray -s torus.yaml` (examples/objects/torus.yaml: JPEG texture) from the scene's directory:
    the PNG equals the oracle's render (PIL-decoded texture) after `as u8` (canvas.rs:98-105)."""
    import sys

    sys.path.insert(0, ROOT)
    from oracle.scene_yaml import build_from_yaml

    root = os.path.join(GOLDEN, "example1")
    out = tmp_path / "torus.png"
    r = _run(["-W", "200", "-H", "100", "-s", "torus.yaml", "-o", str(out), "-a", "1"], cwd=root)
    assert r.returncode == 0, r.stderr
    o, cam = build_from_yaml(open(os.path.join(root, "torus.yaml")).read(), 200, 100, 1, obj_root=root)
    canvas, _ = o.render(cam, max_depth=5)
    ref = np.clip(o.aa_average(canvas, 1) * 255.0, 0, 255).astype(np.uint8)  # f64 as u8 saturates
    got = _png(out)
    diff = int((got != ref).any(axis=2).sum())
    print(f"CLI torus.yaml: {diff} of {got.shape[0] * got.shape[1]} pixels differ from the oracle")
    assert diff == 0

"""Build provenance (rray_amd/build.py): objects are rebuilt by content, not by modification time.  A fake compiler
(a shell script that copies its input to its output and logs the call) stands in for hipcc, so the tests run in
seconds on the CPU and exercise build._compile's real staleness rule on a scratch tree."""
import os
import stat

import pytest

from rray_amd import build as B


@pytest.fixture()
def tree(tmp_path, monkeypatch):
    csrc, obj = tmp_path / "csrc", tmp_path / "obj"
    csrc.mkdir()
    obj.mkdir()
    log = tmp_path / "calls.log"
    cc = tmp_path / "fakecc"
    # copies the source after -c to the path after -o, and logs the source: enough for _compile's bookkeeping
    cc.write_text('#!/bin/sh\nwhile [ $# -gt 0 ]; do case "$1" in -c) src="$2"; shift;; -o) out="$2"; shift;; esac; '
                  f'shift; done\ncp "$src" "$out" && echo "$src" >> "{log}"\n')
    cc.chmod(cc.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(B, "CSRC", str(csrc))
    monkeypatch.setattr(B, "OBJ", str(obj))
    monkeypatch.setattr(B, "HIPCC", str(cc))
    (csrc / "unit.cpp").write_text('#include "dep.hpp"\nint f() { return 1; }\n')
    (csrc / "dep.hpp").write_text("// header v1\n")
    return csrc, obj, log


def _calls(log):
    return open(log).read().count("\n") if os.path.exists(log) else 0


def test_unchanged_sources_are_not_recompiled(tree):
    csrc, obj, log = tree
    deps = [str(csrc / "dep.hpp")]
    out = B._compile("unit.cpp", deps, False)
    assert _calls(log) == 1 and os.path.exists(out) and os.path.exists(out + ".key")
    B._compile("unit.cpp", deps, False)
    assert _calls(log) == 1


def test_edit_with_an_old_mtime_still_recompiles(tree):
    """The case mtimes miss: a source edited and then stamped back in time (a tar / rsync -t restore), older than the
    stale object beside it."""
    csrc, obj, log = tree
    deps = [str(csrc / "dep.hpp")]
    out = B._compile("unit.cpp", deps, False)
    src = csrc / "unit.cpp"
    src.write_text('#include "dep.hpp"\nint f() { return 2; }\n')
    os.utime(src, (1_000_000, 1_000_000))  # 1970: far older than the object
    assert os.path.getmtime(src) < os.path.getmtime(out)
    B._compile("unit.cpp", deps, False)
    assert _calls(log) == 2
    assert open(out).read() == '#include "dep.hpp"\nint f() { return 2; }\n'


def test_header_edit_with_an_old_mtime_recompiles(tree):
    csrc, obj, log = tree
    deps = [str(csrc / "dep.hpp")]
    B._compile("unit.cpp", deps, False)
    hdr = csrc / "dep.hpp"
    hdr.write_text("// header v2\n")
    os.utime(hdr, (1_000_000, 1_000_000))
    B._compile("unit.cpp", deps, False)
    assert _calls(log) == 2


def test_changed_flags_recompile_and_missing_key_recompiles(tree, monkeypatch):
    csrc, obj, log = tree
    deps = [str(csrc / "dep.hpp")]
    out = B._compile("unit.cpp", deps, False)
    monkeypatch.setattr(B, "COMMON", B.COMMON + ["-DEXTRA"])
    B._compile("unit.cpp", deps, False)
    assert _calls(log) == 2
    os.remove(out + ".key")  # an object without a key (e.g. left by an older build script) is never trusted
    B._compile("unit.cpp", deps, False)
    assert _calls(log) == 3


def test_unit_key_covers_source_deps_and_command(tmp_path):
    a, d = tmp_path / "a.cpp", tmp_path / "d.hpp"
    a.write_text("x")
    d.write_text("y")
    k = B.unit_key(str(a), [str(d)], ["cc", "-O3"])
    assert k == B.unit_key(str(a), [str(d)], ["cc", "-O3"])
    assert k != B.unit_key(str(a), [str(d)], ["cc", "-O2"])
    d.write_text("y2")
    assert k != B.unit_key(str(a), [str(d)], ["cc", "-O3"])


def test_in_tree_objects_carry_keys_of_the_current_sources():
    """After build() (conftest builds the library), every product object's key is the content key of the current
    sources: the library that the tests load was linked from exactly these sources."""
    deps = B._dep_files()
    for src in B.SOURCES:
        out = os.path.join(B.OBJ, os.path.splitext(src)[0] + ".o")
        path = os.path.join(B.CSRC, src)
        if src.endswith(".cpp"):
            cmd = [B.HIPCC, "-x", "hip"] + B.COMMON + B.DEVICE + ["-c", path, "-o", out]
        else:
            cmd = [B.HIPCC] + B.COMMON + B.DEVICE + B.UNIT_FLAGS.get(src, []) + ["-c", path, "-o", out] + B.REMARKS
        assert B._key_matches(out, B.unit_key(path, B.unit_deps(path, deps), cmd)), src


def test_unit_deps_follow_includes(tmp_path):
    """A unit depends on what it includes, transitively; an include the scan cannot resolve makes it depend on every
    candidate (conservative)."""
    (tmp_path / "a.hpp").write_text('#include "b.inc"\n')
    (tmp_path / "b.inc").write_text("// leaf\n")
    (tmp_path / "c.hpp").write_text("// unrelated\n")
    u = tmp_path / "u.cpp"
    u.write_text('#include "a.hpp"\n#include <vector>\n')
    cands = [str(tmp_path / n) for n in ("a.hpp", "b.inc", "c.hpp")]
    assert B.unit_deps(str(u), cands) == sorted(cands[:2])
    u.write_text('#include "a.hpp"\n#include "missing.hpp"\n')
    assert B.unit_deps(str(u), cands) == sorted(cands)
    # the product: the chain units depend on the device code, the PNG writer does not
    deps = B._dep_files()
    chain = B.unit_deps(os.path.join(B.CSRC, "render_chain_g0_gl.hip"), deps)
    assert any(d.endswith("device_core.inc") for d in chain)
    png = B.unit_deps(os.path.join(B.CSRC, "png.cpp"), deps)
    assert not any(d.endswith("device_core.inc") for d in png)

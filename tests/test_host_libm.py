"""host_libm.inc (the torus solver's transcendentals on the device) against the host's glibc.

The device build includes the same file with RR_HD = __device__; here it is compiled for the host with g++ and
compared with glibc on seeded random inputs: cbrt is glibc's algorithm restated and must agree on every input;
cos / sin / acos / atan are double-double evaluations rounded once, which agree with glibc except where glibc
itself misses the correct rounding by one ulp (measured 0.01-0.2% of inputs on glibc 2.35)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("libm") / "host_libm_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(HERE, "native", "host_libm_check.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe, "400000"], check=True, capture_output=True, text=True).stdout
    rows = {}
    for line in out.splitlines():
        name, n, diff, far = line.split()
        rows[name] = (int(n), int(diff), int(far))
    return rows


def test_cbrt_is_glibc_bit_for_bit(results):
    for name in ("cbrt", "cbrt_bits"):
        n, diff, _ = results[name]
        assert diff == 0, f"{name}: {diff} of {n} results differ from glibc"


@pytest.mark.parametrize("name", ["cos", "sin", "acos", "acos_ends", "atan"])
def test_rounded_double_double_matches_glibc(results, name):
    n, diff, far = results[name]
    assert far == 0, f"{name}: {far} results differ from glibc by more than one ulp"
    assert diff <= 0.003 * n, f"{name}: {diff} of {n} results differ from glibc"


def test_special_values(results):
    assert results["special"][1] == 0

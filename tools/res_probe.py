"""Register / scratch probe of an edited copy of the sources (no GPU): copies rray_amd/csrc and include/ to a
scratch tree, applies sed scripts, compiles one unit with the product flags and -Rpass-analysis remarks, and prints
the resources of the kernels whose demangled name contains FILTER.
usage: python tools/res_probe.py UNIT.hip FILTER [FILE 'sed script' ...]"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rray_amd import build as B  # noqa: E402


def main():
    unit, flt, edits = sys.argv[1], sys.argv[2], sys.argv[3:]
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(os.path.join(ROOT, "rray_amd", "csrc"), os.path.join(td, "rray_amd", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(td, "include"))
        csrc = os.path.join(td, "rray_amd", "csrc")
        for f, script in zip(edits[::2], edits[1::2]):
            subprocess.run(["sed", "-i", script, os.path.join(csrc, f)], check=True)
        common = [c if not c.startswith("-I") else "-I" + os.path.join(td, "include") for c in B.COMMON]
        cmd = [B.HIPCC] + common + B.DEVICE + B.UNIT_FLAGS.get(unit, []) + B.REMARKS + [
            "-c", os.path.join(csrc, unit), "-o", os.path.join(td, "x.o")]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            sys.exit(1)
        res = B._resources(r.stderr)
        names = sorted(res)
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
        for n, d in zip(names, dem):
            if flt in d:
                print(d[:100], res[n])


if __name__ == "__main__":
    main()

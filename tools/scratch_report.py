"""Per-kernel private-memory (scratch) instructions of the product's device code: compiles each kernel unit to gfx950
assembly (same flags as rray_amd/build.py) and counts scratch_store / scratch_load per kernel, with the source of
every store's surroundings available via --dump.  Scratch stores under a partial exec mask write partial cache lines
that L2 writes back to HBM: the C3 chain kernel's 2.0 GB of writes per frame came from one (render_common.inc
flush_slot).  Usage: python tools/scratch_report.py [unit.hip ...] [--filter SUBSTR] [--dump DIR]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rray_amd import build as B  # noqa: E402


def assemble(unit, out_dir):
    out = os.path.join(out_dir, unit.replace(".hip", ".s"))
    cmd = [B.HIPCC] + B.COMMON + B.DEVICE + B.UNIT_FLAGS.get(unit, []) + ["--cuda-device-only", "-S",
                                                                          os.path.join(B.CSRC, unit), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return out


def kernels(asm_path):
    text = open(asm_path).read()
    parts = re.split(r"\n(_Z\w+):[^\n]*\n", text)
    for i in range(1, len(parts), 2):
        body = parts[i + 1].split(".Lfunc_end")[0]
        yield parts[i], body


def main():
    args = sys.argv[1:]
    flt = None
    dump = None
    if "--filter" in args:
        k = args.index("--filter")
        flt = args[k + 1]
        del args[k:k + 2]
    if "--dump" in args:
        k = args.index("--dump")
        dump = args[k + 1]
        del args[k:k + 2]
    units = args or [u for u in B.SOURCES if u.endswith(".hip")]
    with tempfile.TemporaryDirectory() as td:
        for u in units:
            asm = assemble(u, td)
            names, bodies = [], []
            for n, b in kernels(asm):
                names.append(n)
                bodies.append(b)
            dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
            for n, d, b in zip(names, dem, bodies):
                if flt and flt not in d:
                    continue
                st = len(re.findall(r"^\s+scratch_store", b, re.M))
                ld = len(re.findall(r"^\s+scratch_load", b, re.M))
                print(f"{u:28s} stores {st:3d} loads {ld:3d}  {d[:120]}")
                if dump:
                    os.makedirs(dump, exist_ok=True)
                    open(os.path.join(dump, n[:200] + ".s"), "w").write(b)


if __name__ == "__main__":
    main()

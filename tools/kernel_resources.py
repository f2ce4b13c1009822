"""Register / scratch / occupancy of every kernel in the given render translation units (device-only
compile with -Rpass-analysis=kernel-resource-usage).  Usage:
    python tools/kernel_resources.py [render_levels_g0_gl.hip ...] [--filter shade_kernel] [-D...]
"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rray_amd import build as B  # noqa: E402

KEYS = ["VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]"]


def resources(src, defines):
    cmd = [B.HIPCC] + B.COMMON + B.DEVICE + ["-D" + d for d in defines] + [
        "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(B.CSRC, src), "-o", os.devnull]
    r = subprocess.run(cmd, capture_output=True, text=True)
    out, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(" + "|".join(re.escape(k) for k in KEYS) + r"): (\d+)", line)
        if m and cur:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def main():
    args = sys.argv[1:]
    filt = None
    if "--filter" in args:
        k = args.index("--filter")
        filt = args[k + 1]
        del args[k:k + 2]
    defines = [a[2:] for a in args if a.startswith("-D")]
    srcs = [a for a in args if not a.startswith("-D")] or B.LEVEL_UNITS
    with cf.ThreadPoolExecutor(len(srcs)) as ex:
        res = dict(zip(srcs, ex.map(lambda s: resources(s, defines), srcs)))
    names = [n for r in res.values() for n in r]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    dmap = dict(zip(names, dem))
    print(f"{'kernel':70s} " + " ".join(f"{k.split()[0][:8]:>8s}" for k in KEYS))
    for src, r in res.items():
        for n, v in r.items():
            d = dmap.get(n, n)
            if filt and filt not in d:
                continue
            d = d.replace("rr::", "").replace("(rr::DevScene, rr::LevelArgs)", "").replace("void ", "")
            print(f"{d[:70]:70s} " + " ".join(f"{v.get(k, -1):8d}" for k in KEYS))


if __name__ == "__main__":
    main()

"""Builds the gfx950 render path in-tree: rray_amd/_lib/librray_amd.so and rray_amd/bin/rray.

hipcc (ROCm 7.2) cross-compiles for gfx950 without a GPU.  -ffp-contract=off everywhere: the
reference (rustc) never fuses a*b+c, and bit-parity of every discrete decision depends on it.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIBDIR = os.path.join(HERE, "_lib")
BINDIR = os.path.join(HERE, "bin")
LIB = os.path.join(LIBDIR, "librray_amd.so")
CLI = os.path.join(BINDIR, "rray")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(ROOT, "include")]
DEVICE = ["--offload-arch=" + ARCH, "-mllvm", "-disable-promote-alloca-to-lds"]
LEVEL_UNITS = [f"render_levels_g{g}_{lc}.hip" for g in (2, 1, 0) for lc in ("lds", "gl")]  # slowest first
SOURCES = LEVEL_UNITS + ["render.hip", "api.cpp", "multi.cpp", "flatten.cpp", "frontend.cpp", "yaml.cpp", "png.cpp"]


def _deps_mtime():
    files = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.inc"))
    files += glob.glob(os.path.join(ROOT, "include", "rray", "*.h"))
    files.append(os.path.abspath(__file__))
    return max(os.path.getmtime(f) for f in files)


def _compile(src, deps_mtime, verbose):
    out = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(path), deps_mtime):
        return out
    cmd = [HIPCC] + COMMON + DEVICE + ["-c", path, "-o", out]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip"] + COMMON + DEVICE + ["-c", path, "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return out


def build_variant(name, defines, verbose=False):
    """Experiment build (e.g. RR_STAMPS phase timers) into abtest/<name>/librray_amd.so; select it
    at run time with RRAY_LIB=<path>.  Never used by the product path."""
    out_dir = os.path.join(ROOT, "abtest", name)  # travels to the GPU box (abtest/ is git-ignored)
    os.makedirs(out_dir, exist_ok=True)
    flags = ["-D" + d for d in defines]

    def one(src):
        o = os.path.join(out_dir, os.path.splitext(src)[0] + ".o")
        pre = [HIPCC, "-x", "hip"] if src.endswith(".cpp") else [HIPCC]
        cmd = pre + COMMON + DEVICE + flags + ["-c", os.path.join(CSRC, src), "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stderr}")
        return o

    with cf.ThreadPoolExecutor(min(len(SOURCES), max(1, min(16, os.cpu_count() or 1)))) as ex:
        objs = list(ex.map(one, SOURCES))
    lib = os.path.join(out_dir, "librray_amd.so")
    r = subprocess.run([HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", lib] + objs +
                       ["-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-soname,librray_amd.so"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stderr}")
    return lib


def build(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    dm = _deps_mtime()
    jobs = jobs or min(len(SOURCES), max(1, min(16, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, dm, verbose), SOURCES))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", LIB] + objs + ["-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-soname,librray_amd.so"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    cli_src = os.path.join(CSRC, "cli.cpp")
    if not os.path.exists(CLI) or os.path.getmtime(CLI) < max(os.path.getmtime(LIB), os.path.getmtime(cli_src)):
        cmd = ["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), cli_src, "-o", CLI, "-L" + LIBDIR,
               "-lrray_amd", "-Wl,-rpath,$ORIGIN/../_lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"cli link failed\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        print(build(verbose="-v" in sys.argv))

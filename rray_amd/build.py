"""Builds the gfx950 render path in-tree: rray_amd/_lib/librray_amd.so and rray_amd/bin/rray.

hipcc (ROCm 7.2) cross-compiles for gfx950 without a GPU.  -ffp-contract=off everywhere: the
reference (rustc) never fuses a*b+c, and bit-parity of every discrete decision depends on it.
"""
import concurrent.futures as cf
import glob
import json
import os
import re
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
CHAIN_UNITS = [f"render_chain_g{g}_{lc}.hip" for g in (2, 1, 0) for lc in ("lds", "gl")]
TREE_UNITS = [f"render_tree_g{g}_{lc}.hip" for g in (2, 1, 0) for lc in ("lds", "gl")]
# per-unit flags: the chain kernels' loop must not get loop-invariant constants hoisted into registers (they
# spill instead of being rematerialised)
UNIT_FLAGS = {u: ["-mllvm", "-disable-machine-licm"] for u in CHAIN_UNITS + TREE_UNITS}
# the flat scenes' global-cull level kernels (C2's fused camera kernel): the scheduler's AMDGPU register-pressure
# trackers measured C2 0.1176 -> 0.1166 ms; the same flag on every unit cost C3 and C4 1 % (profiles/r05/ab_trackers.txt)
UNIT_FLAGS["render_levels_g0_gl.hip"] = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
SOURCES = LEVEL_UNITS + CHAIN_UNITS + TREE_UNITS + ["render.hip", "api.cpp", "multi.cpp", "flatten.cpp", "frontend.cpp", "yaml.cpp", "png.cpp", "jpeg.cpp",
                                         "imgfmt.cpp"]


def source_digest():
    """sha256 of the product sources (kernels, host library, header, this build script): identifies
    which build a recorded profile (profiles/pmc_*.json) was measured on."""
    import hashlib

    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*")) + [os.path.join(ROOT, "include", "rray", "rray.h"),
                                                          os.path.abspath(__file__)])
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _dep_files():
    """Every file a unit may include: the csrc headers and .inc files and the public header."""
    files = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.inc"))
    files += glob.glob(os.path.join(ROOT, "include", "rray", "*.h"))
    return sorted(files)


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def unit_deps(path, candidates):
    """The project files `path` includes, transitively (quoted #include lines resolved against the including file's
    directory).  Any quoted include that does not resolve to one of `candidates` makes the unit depend on all of
    them, so a key can only be conservative, never stale."""
    cand = {os.path.realpath(c) for c in candidates}
    seen, todo = set(), [os.path.realpath(path)]
    while todo:
        f = todo.pop()
        with open(f) as fh:
            text = fh.read()
        for inc in _INCLUDE.findall(text):
            q = os.path.realpath(os.path.join(os.path.dirname(f), inc))
            if q not in cand:
                return sorted(candidates)
            if q not in seen:
                seen.add(q)
                todo.append(q)
    return sorted(c for c in candidates if os.path.realpath(c) in seen)


def _sha(paths, extra=""):
    import hashlib

    h = hashlib.sha256(extra.encode())
    for f in paths:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def unit_key(path, deps, cmd):
    """Content key of one object: the unit's source, every file it may include and the compile command.  An object
    is rebuilt whenever its recorded key differs — modification times play no part, so a tree restored with old
    mtimes (tar, rsync -t) next to newer stale objects still recompiles, and a digest match proves the objects came
    from these sources."""
    return _sha([path] + list(deps), "\0".join(cmd))


def _key_file(out):
    return out + ".key"


def _key_matches(out, key):
    kf = _key_file(out)
    return os.path.exists(out) and os.path.exists(kf) and open(kf).read().strip() == key


REMARKS = ["-Rpass-analysis=kernel-resource-usage"]  # per-kernel VGPR / spill report (codegen unchanged)


def _resources(stderr):
    """{mangled kernel name: {"VGPRs": n, "VGPRs Spill": n, ...}} from the resource-usage remarks."""
    out, cur = {}, None
    for line in stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)",
                      line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return out


def cross_lane_kernel(demangled):
    """device_core.inc cross_lane_ok: kernels whose walks read other lanes' registers (v_readlane)."""
    m = re.search(r"rr::(shade_kernel|trace_kernel|n1n2_kernel|shadow_query_kernel|chain_kernel)<([^>]*)>", demangled)
    if not m:
        return False
    args = [a.strip() for a in m.group(2).split(",")]
    g = int(args[0])
    if m.group(1) == "chain_kernel":  # <G, LC, PRE, CP, AR, RM0, RMD>: XL in the flat scenes' kernels only
        return g == 0 and args[3] == "false" and args[4] == "false"
    if m.group(1) == "shade_kernel":  # <G, LC, FUSED, PRE, CP, RM, AR>
        return g < 2 and args[4] == "false" and args[6] == "false"
    return g < 2


def check_cross_lane(resource_files):
    """Fail the build when a cross-lane (XL) kernel spills VGPRs: a register reloaded under a partial exec
    mask keeps stale data in the inactive lanes, and v_readlane would return it (device_core.inc XL)."""
    names, res = [], {}
    for f in resource_files:
        if os.path.exists(f):
            res.update(json.load(open(f)))
    names = sorted(res)
    if not names:
        return []
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    bad = [f"{d} ({res[n].get('VGPRs Spill')} VGPRs spilled)" for n, d in zip(names, dem)
           if cross_lane_kernel(d) and res[n].get("VGPRs Spill", 0) > 0]
    if bad:
        raise RuntimeError("cross-lane kernels must not spill VGPRs (device_core.inc XL); move them to the "
                           "reload path (cross_lane_ok) or lower their register use:\n  " + "\n  ".join(bad))
    return names


def _compile(src, deps, verbose):
    out = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    cmd = [HIPCC] + COMMON + DEVICE + UNIT_FLAGS.get(src, []) + ["-c", path, "-o", out]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip"] + COMMON + DEVICE + ["-c", path, "-o", out]
    else:
        cmd += REMARKS
    key = unit_key(path, unit_deps(path, deps), cmd)
    if _key_matches(out, key) and (src.endswith(".cpp") or os.path.exists(out + ".resources.json")):
        return out
    if os.path.exists(_key_file(out)):
        os.remove(_key_file(out))  # a failed compile leaves no key behind
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    if src.endswith(".hip"):
        json.dump(_resources(r.stderr), open(out + ".resources.json", "w"))
    with open(_key_file(out), "w") as fh:
        fh.write(key + "\n")
    return out


def build_variant(name, defines, verbose=False, patch=None, extra=None):
    """Experiment build into abtest/<name>/librray_amd.so; select it at run time with RRAY_EXPERIMENT=1
    RRAY_LIB=<path>.  Never used by the product path.  patch: a unified diff (tools/patches/*.patch,
    paths relative to the repo root) applied to a copy of the sources (experiment code such as per-wave
    phase timers lives there, not in the product sources); defines: extra -D flags; extra: extra compiler flags
    for the device units (.hip), e.g. a scheduler strategy."""
    import shutil

    out_dir = os.path.join(ROOT, "abtest", name)  # travels to the GPU box (abtest/ is git-ignored)
    os.makedirs(out_dir, exist_ok=True)
    flags = ["-D" + d for d in defines]
    csrc = CSRC
    if patch:
        src_root = os.path.join(out_dir, "src")
        shutil.rmtree(src_root, ignore_errors=True)
        shutil.copytree(os.path.join(ROOT, "rray_amd", "csrc"), os.path.join(src_root, "rray_amd", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src_root, "include"))
        r = subprocess.run(["patch", "-p1", "-s", "-d", src_root, "-i", os.path.abspath(patch)], capture_output=True,
                           text=True)
        if r.returncode != 0:
            raise RuntimeError(f"patch {patch} failed:\n{r.stdout}{r.stderr}")
        csrc = os.path.join(src_root, "rray_amd", "csrc")

    def one(src):
        o = os.path.join(out_dir, os.path.splitext(src)[0] + ".o")
        pre = [HIPCC, "-x", "hip"] if src.endswith(".cpp") else [HIPCC]
        inc = ["-I" + os.path.join(os.path.dirname(os.path.dirname(csrc)), "include")] if patch else []
        cmd = pre + COMMON + inc + DEVICE + UNIT_FLAGS.get(src, []) + flags + ["-c", os.path.join(csrc, src), "-o", o]
        if src.endswith(".hip"):
            cmd += REMARKS + list(extra or [])
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stderr}")
        if src.endswith(".hip"):
            json.dump(_resources(r.stderr), open(o + ".resources.json", "w"))
        return o

    with cf.ThreadPoolExecutor(min(len(SOURCES), max(1, min(16, os.cpu_count() or 1)))) as ex:
        objs = list(ex.map(one, SOURCES))
    # experiment libraries obey the cross-lane rule too: a spilled cross-lane walk reads stale lanes (wrong loop
    # bounds), the likeliest cause of the round-4 teardown hang on an experiment build
    check_cross_lane([o + ".resources.json" for o in objs if os.path.exists(o + ".resources.json")])
    objs.append(_digest_object(verbose, out_dir, "variant-" + name))  # never equal to a source digest
    lib = os.path.join(out_dir, "librray_amd.so")
    r = subprocess.run([HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", lib] + objs +
                       ["-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-soname,librray_amd.so"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stderr}")
    return lib


def _digest_object(verbose=False, out_dir=None, digest=None):
    """The sources' digest baked into the library as rr_build_digest() (build provenance: smoke() and bench.py
    compare it with source_digest() of the tree they run from, so a stale prebuilt .so cannot pass as head).
    Regenerated whenever the digest changes; the library is relinked when this object is newer."""
    d = digest or source_digest()
    out_dir = out_dir or OBJ
    src = os.path.join(out_dir, "build_digest.cpp")
    obj = os.path.join(out_dir, "build_digest.o")
    text = ('// generated by rray_amd/build.py: the product sources\' digest (source_digest())\n'
            f'extern "C" const char* rr_build_digest(void) {{ return "{d}"; }}\n')
    if not os.path.exists(src) or open(src).read() != text:
        open(src, "w").write(text)
    cmd = ["g++", "-O2", "-fPIC", "-c", src, "-o", obj]
    key = unit_key(src, [], cmd)
    if not _key_matches(obj, key):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: build_digest.cpp\n{r.stderr}")
        with open(_key_file(obj), "w") as fh:
            fh.write(key + "\n")
    return obj


def build(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    deps = _dep_files()
    jobs = jobs or min(len(SOURCES), max(1, min(16, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, deps, verbose), SOURCES))
    check_cross_lane([o + ".resources.json" for o in objs if o.endswith(".o") and os.path.exists(o + ".resources.json")])
    objs.append(_digest_object(verbose))
    # the library's key: the link command over the objects' own keys (each the content of its sources)
    cmd = [HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", LIB] + objs + ["-lz", "-L/opt/rocm/lib", "-lrccl", "-Wl,-soname,librray_amd.so"]
    lib_key = _sha([_key_file(o) for o in objs], "\0".join(cmd))
    if not _key_matches(LIB, lib_key):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        with open(_key_file(LIB), "w") as fh:
            fh.write(lib_key + "\n")
    cli_src = os.path.join(CSRC, "cli.cpp")
    cmd = ["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), cli_src, "-o", CLI, "-L" + LIBDIR,
           "-lrray_amd", "-Wl,-rpath,$ORIGIN/../_lib"]
    cli_key = _sha([cli_src, _key_file(LIB)] + unit_deps(cli_src, deps), "\0".join(cmd))
    if not _key_matches(CLI, cli_key):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"cli link failed\n{r.stdout}\n{r.stderr}")
        with open(_key_file(CLI), "w") as fh:
            fh.write(cli_key + "\n")
    return LIB


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":  # variant <name> [--patch file] [--flags "..."] [DEFINE ...]
        args = sys.argv[3:]
        patch, extra = None, None
        while args[:1] in (["--patch"], ["--flags"]):
            if args[0] == "--patch":
                patch = args[1]
            else:
                extra = args[1].split()
            args = args[2:]
        print(build_variant(sys.argv[2], args, patch=patch, extra=extra))
    else:
        print(build(verbose="-v" in sys.argv))

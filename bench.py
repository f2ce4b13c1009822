"""Benchmark: Mpixel-samples/s of the MI355X render path (BASELINE.json metric).

N = 1 (default): BASELINE configs[1] — synthetic 1024-sphere grid + checker plane, point light,
1920x1080, AA=1 (scenes/c2_s1024.yaml).  One step = one frame rendered to the AA-averaged f64 image
in HBM (Camera::render + canvas.rs box average, before `as u8`).  The line also carries the N = 1
value of the multi-GPU workload (`scaling_anchor`), so the 1/2/4/8-GPU curve has its own anchor.

N > 1: BASELINE configs[2] — the same scene at 3840x2160 AA=3, reflective, depth 5 (C3), ONE frame
per step split across the ranks in interleaved 8-row blocks (rank r renders output rows
{y : (y // 8) % N == r}); each rank's f64 AA-averaged tile goes to rank 0 in one RCCL send (the
library's group: one ncclSend per part, one ncclRecv per part into rank 0's staging buffer, one placement
kernel per part), double-buffered so the transfer of frame k overlaps the render of frame k+1 ("scaling": "strong": the frame is fixed).  After the timed region
rank 0 checks that the gathered frame is bit-identical to its own single-part render.
`--mode frames` (opt-in) is the render-farm sharding: one whole frame per rank per step, no
data-path collective ("scaling": "weak").

`python bench.py --gpus N` with no WORLD_SIZE in the environment starts the N ranks itself (a
torch.distributed.run child process, before anything touches the GPU); under torchrun it checks
WORLD_SIZE == N.  `--dry-run` runs the same multi-rank logic on CPU (gloo, the CPU oracle as the
tile renderer at a thumbnail size): a rehearsal of the distributed path, never a measurement.

Also reported: the dominant kernel's roofline (HIP events on the render stream over the timed
region), and the CPU oracle (test-infrastructure restatement of the reference) timed on a bounded
row sample on the host cores, whose rows are also compared with the GPU frame (max |d|).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixel-samples/s (W×H×AA²) at 1/2/4/8 GPUs; max |Δchannel| vs CPU ref"
WORKLOADS = {  # name: (scene, W, H, aa, max_depth)
    "c2_s1024": ("c2_s1024.yaml", 1920, 1080, 1, 5),
    "c3_s1024_reflect": ("c3_s1024_reflect.yaml", 3840, 2160, 3, 5),
    "c4_teapot": ("c4_teapot.yaml", 1920, 1080, 2, 5),
    "c5_area_light": ("c5_area_light.yaml", 1920, 1080, 2, 5),
    "c1_readme": ("c1_readme.yaml", 800, 600, 1, 5),
    # the README's example1.png scene (every shape, CSG, texture, noise): general (G = 2) kernels
    "example1": ("../tests/golden/example1/example1.yaml", 800, 400, 3, 5),
}


def scene_dir(scene_file):
    """Directory a workload's relative OBJ / texture paths resolve against (its YAML's own directory)."""
    return os.path.dirname(os.path.normpath(os.path.join(ROOT, "scenes", scene_file)))
SINGLE_GPU_WORKLOAD = "c2_s1024"      # BASELINE configs[1]
MULTI_GPU_WORKLOAD = "c3_s1024_reflect"  # BASELINE configs[2]
# the library group's partition (--partition): cost-balanced row bands (ABI 10 default) or interleaved 8-row blocks
PARTITION = "bands"
BLOCK = int(os.environ.get("RRAY_BLOCK_ROWS", "8"))  # output rows per interleaved block (env: experiments)
DEPTH_OVERRIDE = None  # --max-depth (experiments only)
# SURVEY.md §8(d) algorithmic flop model (FMA = 2, sqrt/div = 1): per leaf test and per shade event
FLOPS = {"sphere": 57, "plane": 13, "tri": 45, "group": 45, "shade": 250}
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (256 CU x 2.4 GHz x 128 flop/clk), MI355X_MICROARCH.md


def scene_counts(desc):
    kinds = [desc.kind[i] for i in range(desc.n_objects)]
    top = [desc.top[i] for i in range(desc.n_top)]
    return {"sphere": sum(1 for i in top if kinds[i] == 0), "plane": sum(1 for i in top if kinds[i] == 1),
            "group": sum(1 for i in top if kinds[i] == 2), "tri": sum(1 for k in kinds if k in (3, 4)),
            "objects": len(kinds)}


def host_cpu_info():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota when one is set
    (on a shared GPU box nproc shows the whole machine), plus nproc and the lscpu model name."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(math.floor(quota))))
    return {"nproc": os.cpu_count(), "affinity": affinity, "cgroup_quota_cpus": quota, "model": model,
            "threads_used": usable}


def spawn_ranks(args):
    """`bench.py --gpus N` outside torchrun: start N ranks (one process per GPU) as a child
    torch.distributed.run, before any GPU call in this process; exit with its status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 50 for C2-sized frames, 10 for C3)")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help=f"default: {SINGLE_GPU_WORKLOAD} at N=1, {MULTI_GPU_WORKLOAD} at N>1")
    ap.add_argument("--mode", choices=("frames", "tiles"), default=None,
                    help="multi-rank sharding: row tiles of one frame + RCCL transfer (default at N>1) or whole "
                         "frames per rank (opt-in render farm, weak scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-stride", type=int, default=None,
                    help="CPU sample: one 8-row band in every STRIDE bands (default sized to ~10-30 s)")
    ap.add_argument("--no-anchor", action="store_true", help="N=1: skip the C3 scaling anchor")
    ap.add_argument("--no-cold", action="store_true", help="N=1: skip the cold-frame measurements")
    ap.add_argument("--in-flight", type=int, default=1,
                    help="whole-frame steps: frames alternate over this many render contexts and streams (1 = "
                         "one frame at a time, the default: two measured no faster on C2 or C3, "
                         "profiles/r04/pipe_probe.txt; N=1 lines with more also time 1 as `serial`)")
    ap.add_argument("--max-depth", type=int, default=None,
                    help="experiment: override the workload's recursion depth (the line then names it in config)")
    ap.add_argument("--kernel-events", choices=("separate", "timed"), default="separate",
                    help="per-launch HIP events for the roofline: over a second pass of K steps (default) or "
                         "inside the timed region")
    ap.add_argument("--gather", choices=("abi", "torch"), default="abi",
                    help="tiles at N>1: the library's own RCCL group (rr_create_rank + rr_render_gather_device; the "
                         "torch process group only carries host-side coordination over gloo) or torch.distributed's "
                         "per-part RCCL send / receive of the tiles (rray_amd/dist.py FramePipeline)")
    ap.add_argument("--partition", choices=("bands", "interleave"), default="bands",
                    help="tiles at N>1 with --gather abi: cost-balanced row bands received straight into the frame "
                         "(the library default) or interleaved 8-row tiles through a staging buffer and placement "
                         "kernels (RR_PART_INTERLEAVE)")
    ap.add_argument("--force-dist", action="store_true",
                    help="rehearsal: run the multi-rank path (RCCL process group, pipelined gather) even at 1 rank")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank path: gloo, oracle-rendered thumbnail tiles, no GPU")
    args = ap.parse_args()
    global DEPTH_OVERRIDE, PARTITION
    DEPTH_OVERRIDE = args.max_depth
    PARTITION = args.partition

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    mode = args.mode or ("tiles" if world > 1 else "frames")
    workload = args.workload or (MULTI_GPU_WORKLOAD if world > 1 and mode == "tiles" else SINGLE_GPU_WORKLOAD)
    if args.dry_run:
        return dry_run(args, world, mode, workload)
    return gpu_bench(args, world, mode, workload)


class Contexts:
    """The render contexts a Session alternates its frames over, seen as one for profiling and statistics."""

    def __init__(self, rends):
        self.rends = rends
        self.last = 0  # the context that rendered the latest frame

    def kernel_profile(self, enable):
        for r in self.rends:
            r.kernel_profile(enable)

    def kernel_times(self):
        out = {}
        for r in self.rends:
            for k, (ms, n) in r.kernel_times().items():
                a, b = out.get(k, (0.0, 0))
                out[k] = (a + ms, b + n)
        return out

    def last_stats(self):
        return self.rends[self.last].last_stats()


class Session:
    """One workload on this rank: the scene in HBM and a `step()` that renders one frame (frames mode /
    one part) or this rank's tile of one frame plus the pipelined gather (tiles mode).

    in_flight (one part): consecutive frames alternate over that many render contexts (scene copy +
    workspace each) on as many streams, each into its own output buffer, so frame k+1's waves fill the GPU
    while frame k's last waves finish — how a renderer serving a stream of frames uses the library (the
    multi-GPU group does the same per part).  Every step still renders one whole frame."""

    def __init__(self, R, workload, dev, local, rank, world, tiles, distributed, rend, gather="abi", in_flight=1):
        import torch
        from rray_amd import dist as rdist

        self.workload = workload
        self.scene_file, self.W, self.H, self.aa, self.depth = WORKLOADS[workload]
        if DEPTH_OVERRIDE is not None:
            self.depth = DEPTH_OVERRIDE
        self.text = open(os.path.join(ROOT, "scenes", self.scene_file)).read()
        self.scene = R.YamlScene(self.text, self.W, self.H, self.aa, obj_root=scene_dir(self.scene_file))
        self.counts = scene_counts(self.scene.desc())
        self.rend = rend
        rend.upload(self.scene)
        self.cam = self.scene.camera
        self.dev = dev
        self.tiles = tiles
        self.multi = distributed and tiles
        self.gather = gather
        self.rank = rank
        self.pipe = None
        self.tile = None
        self.frame_t = None
        part, nparts = (rank, world) if tiles else (0, 1)
        rows = R.part_rows(self.H, part, nparts, BLOCK)
        self.k = 0
        self.slots = None
        if not self.multi:
            # the AA-averaged f64 image (the drop-in's Canvas, before `as u8`)
            self.tile = torch.zeros((len(rows), self.W, 3), dtype=torch.float64, device=dev)
            self.opts = R._lib.RenderOpts(self.aa, self.depth, 0, 0, part, nparts, BLOCK,
                                          R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
            self.stream = torch.cuda.current_stream(dev)
            if in_flight > 1:
                extra = [R.Renderer(local) for _ in range(in_flight - 1)]
                for r in extra:
                    r.upload(self.scene)
                self.slots = [(r, torch.cuda.Stream(dev), self.tile if i == 0 else torch.zeros_like(self.tile))
                              for i, r in enumerate([rend] + extra)]
                self.extra = extra
                self.rend = Contexts([rend] + extra)
        elif gather == "abi":
            # the library's group context splits the frame into this rank's row tile, gathers the f64
            # tiles to rank 0 with one RCCL send / receive per part (double-buffered: frame k+1 renders while frame k is
            # gathered) and un-interleaves them into frame_t
            if rank == 0:
                self.frame_t = torch.zeros((self.H, self.W, 3), dtype=torch.float64, device=dev)
            self.opts = R._lib.RenderOpts(self.aa, self.depth, 0, 0, 0, 1, BLOCK,
                                          R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING |
                                          (R._lib.RR_PART_INTERLEAVE if PARTITION == "interleave" else 0))
            self.stream = torch.cuda.current_stream(dev)
        else:
            # f64 tiles (bit-identical to the 1-GPU image), double-buffered: rendering frame k+1 overlaps
            # the per-part RCCL transfer of frame k
            self.pipe = rdist.FramePipeline(self.H, self.W, 3, torch.float64, dev, block=BLOCK)
            self.opts = R._lib.RenderOpts(self.aa, self.depth, 0, 0, rank, world, BLOCK,
                                          R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
            self.stream = torch.cuda.Stream(dev)

    def step(self):
        import torch

        if not self.multi:
            if self.slots:
                j = self.k % len(self.slots)
                r, st, out = self.slots[j]
                r.render_device(self.cam, self.opts, None, out.data_ptr(), st.cuda_stream)
                self.rend.last = j
                self.k += 1
                return
            self.rend.render_device(self.cam, self.opts, None, self.tile.data_ptr(), self.stream.cuda_stream)
            return
        if self.gather == "abi":
            self.rend.render_gather_device(self.cam, self.opts, self.frame_t.data_ptr() if self.rank == 0 else None,
                                           self.stream.cuda_stream)
            return
        i, buf, prev = self.pipe.acquire()
        with torch.cuda.stream(self.stream):
            if prev is not None:
                prev.wait()  # the gather that last read this buffer
            self.rend.render_device(self.cam, self.opts, None, buf.data_ptr(), self.stream.cuda_stream)
        torch.cuda.current_stream(self.dev).wait_stream(self.stream)
        self.pipe.submit(i)

    def frame(self):
        """The latest assembled AA-averaged frame (rank 0 in tiles mode), as a CPU numpy array."""
        if self.multi and self.gather == "abi":
            return self.frame_t.cpu().numpy() if self.frame_t is not None else None
        if self.multi:
            return self.pipe.frame.cpu().numpy() if self.pipe.frame is not None else None
        if self.slots:
            return self.slots[(self.k - 1) % len(self.slots)][2].cpu().numpy()
        return self.tile.cpu().numpy()

    def close(self):
        for r in getattr(self, "extra", []):
            r.close()


def timed_loop(sess, steps, warmup, distributed, dist, torch, kernel_events="separate"):
    def sync():
        if sess.pipe is not None:
            sess.pipe.drain()
        torch.cuda.synchronize(sess.dev)
        if distributed:
            dist.barrier()

    for _ in range(warmup):
        sess.step()
    sync()
    # Per-launch HIP events cost ~5 % of a C2 frame, so by default the timed region runs without them
    # and the dominant kernel's launches are timed with HIP events (render stream) over a second pass
    # of the same K steps right after it; --kernel-events timed puts them inside the timed region.
    in_region = kernel_events == "timed"
    sess.rend.kernel_profile(in_region)
    t0 = time.perf_counter()
    for _ in range(steps):
        sess.step()
    t_enq = time.perf_counter()
    sync()
    t1 = time.perf_counter()
    if not in_region:
        sess.rend.kernel_profile(True)
        for _ in range(steps):
            sess.step()
        sync()
    ktimes = sess.rend.kernel_times()
    sess.rend.kernel_profile(False)
    stats = sess.rend.last_stats()
    elapsed = t1 - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.to(sess.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, (t_enq - t0), ktimes, stats, in_region


def roofline_of(sess, ktimes, stats, steps, in_region):
    ktimes = {k: v for k, v in ktimes.items() if v[1]}
    if not ktimes:
        ktimes = {"none": (0.0, 1)}
    dom = max(ktimes, key=lambda k: ktimes[k][0])
    dom_ms, dom_n = ktimes[dom]
    if dom in ("chain", "deep"):  # the chain kernels' two launches share one flop count (every walk of the frame)
        dom = "chain"
        dom_ms = sum(ktimes[k][0] for k in ("chain", "deep") if k in ktimes)
        dom_n = ktimes["chain"][1] if "chain" in ktimes else dom_n
    # f64 flops this kernel executed in the last step: the exact leaf tests its walks ran after culling
    # (trace / n1n2 walks; the shade kernel runs the is_shadowed walks) + the shade-event model
    ef = stats["exact_flops"]
    flops = {"trace": ef[0], "n1n2": ef[2], "shade": ef[1] + stats["shade_events"] * FLOPS["shade"],
             "trace_shade": ef[0] + ef[1] + stats["shade_events"] * FLOPS["shade"],
             "chain": ef[0] + ef[1] + stats["shade_events"] * FLOPS["shade"]}.get(dom, 0)
    launches_per_step = dom_n / steps
    # flops of one step / (this kernel's time per step) == per-launch flops / average launch duration
    achieved = flops / (dom_ms / steps / 1e3) / 1e12 if dom_ms > 0 else 0.0
    # HBM traffic and VALU busy come from a RECORDED rocprofv3 PMC session (profiles/pmc_<workload>.json; PMC
    # counters need their own profiler runs).  They are reported only when that session measured this very
    # build (same source digest); otherwise null, with the recorded values kept under "recorded_profile".
    from rray_amd.build import source_digest

    traffic, entry, rec = None, {}, {"status": "none"}
    pmc = os.path.join(ROOT, "profiles", f"pmc_{sess.workload}.json")
    if os.path.exists(pmc):
        try:
            per_kernel = json.load(open(pmc))
            # the fused trace+shade launch is the shade_kernel<..., FUSED> instantiation in rocprof's naming
            entry = per_kernel.get(dom) or (per_kernel.get("shade") if dom == "trace_shade" else None) or {}
        except (OSError, ValueError):
            entry = {}
        here = source_digest()
        current = bool(entry) and entry.get("src_digest") == here
        rec = {"status": "current" if current else "stale", "profile": entry.get("profile"),
               "profile_src_digest": entry.get("src_digest"), "this_build_src_digest": here,
               "hbm_bytes_per_launch": entry.get("hbm_bytes_per_launch"), "valu_busy_frac": entry.get("valu_busy_frac")}
        if current:
            traffic = entry.get("hbm_bytes_per_launch")
        else:
            entry = {}
    c = sess.counts
    # SURVEY §8(d) full-scan model for the same rays: what the reference's algorithm would execute
    per_ray = FLOPS["sphere"] * c["sphere"] + FLOPS["plane"] * c["plane"] + FLOPS["group"] * c["group"] + FLOPS["tri"] * c["tri"]
    ref_flops = {"trace": stats["rays"] * per_ray, "n1n2": stats["n1n2_scans"] * per_ray,
                 "shade": stats["shadow_rays"] * per_ray + stats["shade_events"] * FLOPS["shade"],
                 "trace_shade": (stats["rays"] + stats["shadow_rays"]) * per_ray + stats["shade_events"] * FLOPS["shade"],
                 "chain": (stats["rays"] + stats["shadow_rays"]) * per_ray + stats["shade_events"] * FLOPS["shade"]
                 }.get(dom, 0)
    ref_tf = ref_flops / (dom_ms / steps / 1e3) / 1e12 if dom_ms > 0 else 0.0
    return {"bound": "valu_fp64", "achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP64_PEAK_TFLOPS, 4), "traffic": traffic, "kernel": dom,
            "kernel_ms": round(dom_ms / dom_n, 4),
            "kernel_timing": "HIP events around every launch on the render stream, "
                             + ("inside the timed region" if in_region else
                                f"over a second pass of the same {steps} steps after the timed region"),
            "launches_per_step": launches_per_step,
            "flops_per_launch": flops / launches_per_step if launches_per_step else 0,
            "reference_equivalent": {"tflops": round(ref_tf, 2), "frac": round(ref_tf / FP64_PEAK_TFLOPS, 3),
                                     "flops_per_step": ref_flops,
                                     "model": "SURVEY §8(d) full scan (every ray tests every primitive; "
                                              "triangles counted as if their group box were hit)"},
            "traffic_source": "recorded rocprofv3 PMC session of this build (2*FETCH_SIZE + WRITE_SIZE per launch)"
                              if traffic is not None else "no PMC session of this build recorded: null",
            "recorded_profile": rec,
            "valu_busy": {"frac": entry.get("valu_busy_frac"), "rocprof_kernel_ms":
                          (entry["rocprof_avg_ns"] / 1e6 if entry.get("rocprof_avg_ns") else None),
                          "source": entry.get("profile"),
                          "model": "SQ_ACTIVE_INST_VALU (quad-cycles) x SQ_WAVES x 4 / (1024 SIMDs x 2.4 GHz x "
                                   "rocprof mean launch time): the share of all SIMD cycles issuing vector "
                                   "instructions"},
            "note": "bound = FP64 vector ALU (no MFMA: no dense contraction on this path; HBM idle). achieved = f64 "
                    "flops the kernel executed: exact leaf tests after culling (SURVEY §8d model: sphere 57, plane 13, "
                    "triangle/group 45) + 250 per shade event, / kernel time; the f32 bundle/line culling that removes "
                    "the other tests is overhead, not counted. Peak = MI355X FP64 vector 78.6 TF; bit-parity forbids "
                    "FMA contraction (DESIGN.md §4)"}


def default_cpu_stride(workload):
    # bounded oracle sample (~10-30 s on 16 cores): every band for the small frames, one 8-row band in
    # every K for the big ones
    return {"c2_s1024": 1, "c1_readme": 1, "c4_teapot": 4, "c5_area_light": 16, "c3_s1024_reflect": 16,
            "example1": 4}[workload]


def cpu_leg(sess, args, gpu_img):
    """The oracle on the host cores over a bounded band sample of the same frame, and the GPU frame's
    rows compared with it (test-infrastructure checker; nothing here is measured as the product)."""
    import numpy as np

    import oracle
    from oracle.scene_yaml import build_from_yaml

    info = host_cpu_info()
    threads = info["threads_used"]
    stride = args.cpu_stride or default_cpu_stride(sess.workload)
    W, H, aa = sess.W, sess.H, sess.aa
    o, ocam = build_from_yaml(sess.text, W, H, aa, obj_root=scene_dir(sess.scene_file))
    tc = time.perf_counter()
    canvas, _ = o.render(ocam, max_depth=sess.depth, threads=threads, band=BLOCK * aa, band_stride=stride)
    dt = time.perf_counter() - tc
    sel = np.array([y for y in range(H * aa) if (y // (BLOCK * aa)) % stride == 0])
    cpu_samples = len(sel) * W * aa
    cpu = {"value": round(cpu_samples / dt / 1e6, 5), "unit": "Mpixel-samples/s", "cores": threads, "kind": "port",
           "host": info,
           "sample": f"oracle (C++ restatement, reference structure: per-object inverse, full xs list + stable "
                     f"sort, recursion; {threads} threads) on {len(sel) // aa} of {H} output rows of "
                     f"{sess.workload} (one {BLOCK}-row band in every {stride}), {cpu_samples} samples, {dt:.1f}s"}
    avg = o.aa_average(np.nan_to_num(canvas), aa)
    del canvas
    out_rows = sorted(set(int(y) // aa for y in sel))
    d = np.abs(gpu_img[out_rows] - avg[out_rows])
    parity = {"workload": sess.workload, "rows_checked": len(out_rows), "max_abs_diff": float(np.max(d)),
              "bit_exact_frac": float(np.mean(gpu_img[out_rows] == avg[out_rows])),
              "u8_pixels_different": int(np.sum(np.any(o.quantize(gpu_img[out_rows]) != o.quantize(avg[out_rows]),
                                                        axis=-1)))}
    return cpu, parity


def cold_frames(R, workload, dev, local, torch):
    """The single-shot cost the warm loop hides (the reference renders once per invocation: main.rs:73-77 ->
    scene_builder_yaml.rs:408).  `fresh_context_ms`: a new context with the scene uploaded (untimed), its first
    frame — workspace allocation, the per-tile camera bundles, and for group scenes the launch-order frame plus
    the tile-order sort; `new_camera_ms`: a warm context's first frame of a moved camera (bundles recomputed);
    `warm_ms`: the frame after it.  Host wall clock around each frame with a device synchronise."""
    import ctypes

    scene_file, W, H, aa, depth = WORKLOADS[workload]
    text = open(os.path.join(ROOT, "scenes", scene_file)).read()
    scene = R.YamlScene(text, W, H, aa, obj_root=scene_dir(scene_file))
    r = R.Renderer(local)
    r.upload(scene)
    out = torch.zeros((H, W, 3), dtype=torch.float64, device=dev)
    opts = R._lib.RenderOpts(aa, depth, 0, 0, 0, 1, BLOCK, R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)
    st = torch.cuda.current_stream(dev)

    def frame(cam):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.render_device(cam, opts, None, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3

    cam = scene.camera
    first = frame(cam)
    warm0 = frame(cam)
    moved = type(cam)()
    ctypes.pointer(moved)[0] = cam
    moved.transform[3] += 1e-3  # a slightly moved camera: a new view transform, so new tile bundles
    new_cam = frame(moved)
    warm = frame(moved)
    r.close()
    # a second fresh context in the same process: its first frame without the process's one-time code-object load
    r = R.Renderer(local)
    r.upload(scene)
    again = frame(cam)
    r.close()
    return {"workload": workload, "fresh_context_ms": round(first, 4), "second_frame_ms": round(warm0, 4),
            "new_camera_ms": round(new_cam, 4), "warm_ms": round(warm, 4), "fresh_context_again_ms": round(again, 4),
            "note": "host wall clock of one frame with a device synchronise on both sides (launch latency "
                    "included): first frame of a new context (workspace allocation; the first such frame of the "
                    "process also loads the kernels' code objects), then a moved camera on the warm context, then "
                    "the first frame of a second new context"}


def gpu_bench(args, world, mode, workload):
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    distributed = world > 1 or args.force_dist
    tiles = mode == "tiles"
    abi_group = distributed and tiles and args.gather == "abi"
    if distributed and "RANK" not in os.environ:  # --force-dist outside torchrun: a 1-rank group
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
    if distributed:
        if abi_group:  # RCCL lives in the library; the process group only coordinates the hosts
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import rray_amd as R

    # build provenance: the library must be the build of this tree's sources (rr_build_digest)
    lib_digest, src_digest = R._lib.check_provenance()
    dev = torch.device("cuda", local)
    torch.zeros(1, device=dev)  # torch's HIP runtime initialises first (the library shares it)
    if abi_group:
        uid = [R.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        rend = R.Renderer.rank(local, world, rank, uid[0])
    else:
        rend = R.Renderer(local)
    in_flight = max(1, args.in_flight)
    sess = Session(R, workload, dev, local, rank, world, tiles, distributed, rend, args.gather, in_flight)
    big = WORKLOADS[workload][1] * WORKLOADS[workload][2] * WORKLOADS[workload][3] ** 2 > 20_000_000
    steps = args.steps if args.steps is not None else (10 if big else 50)
    warmup = args.warmup if args.warmup is not None else (2 if big else 10)
    elapsed, t_enq, ktimes, stats, in_region = timed_loop(sess, steps, warmup, distributed, dist, torch,
                                                          args.kernel_events)
    samples_per_frame = sess.W * sess.H * sess.aa * sess.aa
    frames_per_step = world if not tiles else 1  # frames mode: every rank renders a whole frame per step
    value = frames_per_step * samples_per_frame * steps / elapsed / 1e6
    roofline = roofline_of(sess, ktimes, stats, steps, in_region)

    # tiles: the gathered frame must be bit-identical to one part rendering the whole frame (§8(e)); rank 0
    # also times that single-GPU render of the same workload (the other ranks wait at the barrier), so the
    # line carries its own 1-GPU point
    identity = single = None
    if sess.multi:
        gathered = sess.frame() if rank == 0 else None
        if rank == 0:
            one = R.Renderer(local)  # a plain single-device context renders the whole frame as one part
            one.upload(sess.scene)
            full = one.render(sess.cam, aa=sess.aa, max_depth=sess.depth)["avg"]
            identity = {"bit_identical_to_1_part": bool(np.array_equal(gathered, full)),
                        "max_abs_diff": float(np.max(np.abs(gathered - full)))}
            a = Session(R, workload, dev, local, 0, 1, True, False, one, in_flight=in_flight)
            k1 = max(2, min(steps, 5))
            a_el, _, _, _, _ = timed_loop(a, k1, 1, False, dist, torch)
            single = {"n_gpus": 1, "steps": k1, "ms_per_step": round(a_el / k1 * 1e3, 4),
                      "value": round(a.W * a.H * a.aa * a.aa * k1 / a_el / 1e6, 3), "frames_in_flight": in_flight,
                      "note": "the same frame rendered as one part on rank 0's GPU after the timed region"}
            a.close()
            one.close()
        dist.barrier()

    cpu = parity = anchor = cold = serial = None
    if rank == 0 and world == 1 and not args.force_dist and sess.slots:
        # the same frames one at a time (one context, one stream): the per-frame latency a single render sees
        ser = Session(R, workload, dev, local, 0, 1, tiles, False, rend)
        s_el, _, s_kt, _, _ = timed_loop(ser, steps, warmup, False, dist, torch)
        serial = {"frames_in_flight": 1, "steps": steps, "ms_per_step": round(s_el / steps * 1e3, 4),
                  "value": round(samples_per_frame * steps / s_el / 1e6, 3),
                  "kernels_ms_per_step": {k: round(v[0] / steps, 4) for k, v in s_kt.items() if v[1]}}
    if rank == 0 and world == 1 and not args.force_dist and not args.no_cold:
        cold = [cold_frames(R, w, dev, local, torch) for w in dict.fromkeys([workload, "c4_teapot"])]
    if rank == 0 and world == 1 and not args.force_dist:
        if not args.no_cpu_baseline:
            cpu, parity = cpu_leg(sess, args, sess.frame())
        if not args.no_anchor and workload != MULTI_GPU_WORKLOAD:
            # the N = 1 point of the multi-GPU curve: C3 as one part on this GPU
            a = Session(R, MULTI_GPU_WORKLOAD, dev, local, 0, 1, True, False, rend, in_flight=in_flight)
            a_el, _, _, _, _ = timed_loop(a, 5, 1, False, dist, torch)
            a.close()
            a_samples = a.W * a.H * a.aa * a.aa
            anchor = {"workload": MULTI_GPU_WORKLOAD, "n_gpus": 1, "value": round(a_samples * 5 / a_el / 1e6, 3),
                      "ms_per_step": round(a_el / 5 * 1e3, 4), "steps": 5, "warmup": 1, "frames_in_flight": in_flight,
                      "note": "N=1 value of the N>1 workload (row tiles with nparts=1), for the scaling curve"}
    if rank == 0:
        via = ("library RCCL group: rr_create_rank + rr_render_gather_device" if args.gather == "abi" else
               "torch.distributed RCCL isend / irecv per part")
        part_kind = ("cost-balanced row bands" if PARTITION == "bands" else "interleaved 8-row tiles") \
            if args.gather == "abi" else "interleaved 8-row tiles"
        par = (f"{part_kind} x{world} + rccl send/recv per part (f64 tiles, pipelined; {via})" if world > 1 or sess.multi else
               "single GPU, whole frame") if tiles else \
            f"frame-parallel x{world} (one whole frame per rank per step, no data-path collective)"
        line = {"metric": METRIC, "value": round(value, 3), "unit": "Mpixel-samples/s", "n_gpus": world,
                "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
                "higher_is_better": True,
                "scaling": "strong" if tiles else "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic (scenes/make_scenes.py, seeded)",
                "config": {"workload": workload, "scene": sess.scene_file, "width": sess.W, "height": sess.H,
                           "aa": sess.aa, "max_depth": sess.depth, "samples_per_step": samples_per_frame,
                           "objects": sess.counts["objects"], "frames_per_step": frames_per_step,
                           "parallelism": par},
                "roofline": roofline, "cpu_baseline": cpu, "parity_sample": parity, "cold_frames": cold,
                "build": {"library_digest": lib_digest, "source_digest": src_digest, "match": lib_digest == src_digest},
                "frames_in_flight": 2 if sess.multi and args.gather == "abi" else len(sess.slots or [0]),
                "serial": serial,
                "tile_identity": identity, "scaling_anchor": anchor, "single_gpu": single,
                "bands": sess.rend.bands() if sess.multi and args.gather == "abi" else None,
                "speedup_vs_single_gpu": round(value / single["value"], 3) if single else None,
                "kernels_ms_per_step": {k: round(v[0] / steps, 4) for k, v in ktimes.items() if v[1]},
                "host_enqueue_ms_per_step": round(t_enq / steps * 1e3, 4),
                "stats_last_step": {k: stats[k] for k in ("rays", "shadow_rays", "shade_events", "n1n2_scans",
                                                          "prim_tests", "exact_flops", "wave_visits")}}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    sess.close()
    rend.close()


def dry_run(args, world, mode, workload):
    """CPU rehearsal of the multi-rank bench (gloo): same spawn, world check, row partition, pipelined
    gather and max-over-ranks timing; each rank's tile is rendered by the CPU oracle at a thumbnail size
    (test infrastructure standing in for the GPU).  Not a measurement."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from oracle.scene_yaml import build_from_yaml
    from rray_amd import dist as rdist

    rank = int(os.environ.get("RANK", "0"))
    distributed = world > 1
    if distributed:
        dist.init_process_group("gloo")
    tiles = mode == "tiles"
    scene_file, W0, H0, aa, depth = WORKLOADS[workload]
    W, H = 96, 54
    text = open(os.path.join(ROOT, "scenes", scene_file)).read()
    o, cam = build_from_yaml(text, W, H, aa, obj_root=scene_dir(scene_file))
    steps = args.steps or 2
    part, nparts = (rank, world) if tiles else (0, 1)
    rows = rdist.tile_rows(H, part, nparts, BLOCK)

    def render_tile(out):
        canvas, _ = o.render(cam, max_depth=depth, threads=2, band=BLOCK * aa, band_stride=nparts, band_phase=part)
        avg = o.aa_average(np.nan_to_num(canvas), aa)
        out[: len(rows)] = torch.from_numpy(avg[rows])

    # multi.cpp's layout: unpadded f64 tiles, one send per part to rank 0, received back to back into a staging
    # buffer (part p at rr_stage_row_offset) and placed by the library's rr_unshuffle_host (the runs the device
    # placement kernels move)
    pipe = rdist.FramePipeline(H, W, 3, torch.float64, torch.device("cpu"), block=BLOCK) if (tiles and distributed) \
        else None
    t0 = time.perf_counter()
    for _ in range(steps):
        if pipe is not None:
            i, buf, prev = pipe.acquire()
            if prev is not None:
                prev.wait()
            render_tile(buf)
            pipe.submit(i)
        else:
            render_tile(torch.zeros((len(rows), W, 3), dtype=torch.float64))
    if pipe is not None:
        pipe.drain()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    identity = None
    if pipe is not None:  # one more frame through the library's host un-interleave (rr_unshuffle_host)
        tile = torch.zeros((len(rows), W, 3), dtype=torch.float64)
        render_tile(tile)
        via_lib = rdist.gather_frame(tile, H, BLOCK)
    if rank == 0 and pipe is not None:
        full, _ = o.render(cam, max_depth=depth, threads=2)
        ref = o.aa_average(np.nan_to_num(full), aa)
        identity = {"bit_identical_to_1_part": bool(np.array_equal(pipe.frame.numpy(), ref)),
                    "rr_unshuffle_host_bit_identical": bool(np.array_equal(via_lib.numpy(), ref)),
                    "layout": "multi.cpp: unpadded f64 tiles, one send / receive per part into the staging "
                              "buffer at rr_stage_row_offset, library run placement (rr_unshuffle_host)"}
    if rank == 0:
        frames_per_step = world if not tiles else 1
        line = {"metric": METRIC, "value": round(frames_per_step * W * H * aa * aa * steps / elapsed / 1e6, 6),
                "unit": "Mpixel-samples/s", "n_gpus": world, "steps": steps, "warmup": 0,
                "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True,
                "scaling": "strong" if tiles else "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic (scenes/make_scenes.py, seeded)",
                "dry_run": f"gloo on CPU, CPU-oracle tiles at {W}x{H} (not {W0}x{H0}): a rehearsal, not a measurement",
                "config": {"workload": workload, "scene": scene_file, "width": W, "height": H, "aa": aa,
                           "max_depth": depth, "frames_per_step": frames_per_step,
                           "parallelism": (f"row-tiles x{world} + per-part send/recv (f64 tiles, pipelined)" if tiles else
                                           f"frame-parallel x{world} (one whole frame per rank per step, "
                                           "no data-path collective)")},
                "tile_identity": identity}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

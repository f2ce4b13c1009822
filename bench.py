"""Benchmark: Mpixel-samples/s of the MI355X render path on BASELINE.json's single-GPU config.

Workload (configs[1]): synthetic 1024-sphere grid + checker plane, point light, 1920x1080, AA=1
(scenes/c2_s1024.yaml).  One step = one frame rendered to the AA-averaged f64 image in HBM
(Camera::render + canvas.rs box average, before `as u8`).

With N ranks (torchrun, one process per GPU) there are two shardings:
* --mode frames (default): the job renders a batch of N frames per step, one whole C2 frame per
  rank, each kept resident on its rank (a renderer farm's frame sharding).  No data-path collective;
  the process group only carries the barrier and the max-over-ranks timing ("scaling": "weak").
* --mode tiles: one frame per step, its rows split in interleaved 8-row blocks; the tiles (f32) are
  gathered to rank 0 with one RCCL gather per step, double-buffered so the gather of frame k overlaps
  the render of frame k+1 ("scaling": "strong": the frame is fixed).  North_star's C3 layout.

Also reported: the dominant kernel's roofline (HIP events on the render stream over the timed
region), and the CPU oracle (test-infrastructure restatement of the reference) timed on a bounded
row sample on the host cores, whose rows are also compared with the GPU frame (max |d|).
"""
import argparse
import json
import os
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
}
# SURVEY.md §8(d) algorithmic flop model (FMA = 2, sqrt/div = 1): per leaf test and per shade event
FLOPS = {"sphere": 57, "plane": 13, "tri": 45, "group": 45, "shade": 250}
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 MFMA dense) peak, MI355X_MICROARCH.md / SURVEY §8d


def scene_counts(desc):
    kinds = [desc.kind[i] for i in range(desc.n_objects)]
    top = [desc.top[i] for i in range(desc.n_top)]
    return {"sphere": sum(1 for i in top if kinds[i] == 0), "plane": sum(1 for i in top if kinds[i] == 1),
            "group": sum(1 for i in top if kinds[i] == 2), "tri": sum(1 for k in kinds if k in (3, 4)),
            "objects": len(kinds)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # a C2 step is ~0.18 ms: 50 + 10 frames settle the clocks
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c2_s1024", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-stride", type=int, default=1, help="CPU sample: one 8-row band in every STRIDE bands")
    ap.add_argument("--mode", choices=("frames", "tiles"), default="frames",
                    help="multi-rank sharding: whole frames per rank (weak) or row tiles of one frame + RCCL gather")
    ap.add_argument("--kernel-events", choices=("separate", "timed"), default="separate",
                    help="per-launch HIP events for the roofline: over a second pass of K steps (default) or "
                         "inside the timed region")
    ap.add_argument("--force-dist", action="store_true",
                    help="rehearsal: run the multi-rank path (RCCL process group, pipelined gather) even at 1 rank")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    distributed = world > 1 or args.force_dist
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    tiles = args.mode == "tiles"
    multi = distributed and tiles  # row tiles + pipelined gather; frames mode renders like one GPU

    import rray_amd as R

    scene_file, W, H, aa, depth = WORKLOADS[args.workload]
    text = open(os.path.join(ROOT, "scenes", scene_file)).read()
    scene = R.YamlScene(text, W, H, aa, obj_root=os.path.join(ROOT, "scenes"))
    counts = scene_counts(scene.desc())
    rend = R.Renderer(local)
    rend.upload(scene)
    cam = scene.camera
    block = 8
    part, nparts = (rank, world) if tiles else (0, 1)
    rows = R.part_rows(H, part, nparts, block)
    dev = torch.device("cuda", local)
    from rray_amd import dist as rdist
    if not multi:
        # the AA-averaged f64 image (the drop-in's Canvas, before `as u8`)
        tile = torch.zeros((len(rows), W, 3), dtype=torch.float64, device=dev)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, part, nparts, block, R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING)

        side = torch.cuda.Stream(dev) if os.environ.get("RRAY_BENCH_SIDE_STREAM") else None

        def step():
            stream = (side or torch.cuda.current_stream(dev)).cuda_stream
            rend.render_device(cam, opts, None, tile.data_ptr(), stream)
    else:
        # tiles travel as f32 (the f64 average rounded once; far inside the 1e-5 gate), double-buffered
        # so that rendering frame k+1 overlaps the RCCL gather of frame k
        pipe = rdist.FramePipeline(H, W, 3, torch.float32, dev, block=block)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, rank, world, block,
                                 R._lib.RR_OUT_AVG_F32 | R._lib.RR_NO_FRAME_TIMING)
        render_stream = torch.cuda.Stream(dev)

        trace_host = {} if os.environ.get("RRAY_BENCH_TRACE") else None

        def lap(name, t):
            if trace_host is None:
                return t
            now = time.perf_counter()
            trace_host[name] = trace_host.get(name, 0.0) + now - t
            return now

        def step():
            t = time.perf_counter()
            i, buf, prev = pipe.acquire()
            with torch.cuda.stream(render_stream):
                if prev is not None:
                    prev.wait()  # the gather that last read this buffer
                t = lap("prev.wait", t)
                rend.render_device(cam, opts, None, buf.data_ptr(), render_stream.cuda_stream)
                t = lap("render_device", t)
            torch.cuda.current_stream(dev).wait_stream(render_stream)
            t = lap("wait_stream", t)
            pipe.submit(i)
            lap("submit", t)
        tile = None

    def sync():
        if multi:
            pipe.drain()
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    sync()
    if multi and trace_host is not None:
        trace_host.clear()
    # Per-launch HIP events cost ~5 % of a C2 frame, so by default the timed region runs without them
    # and the dominant kernel's launches are timed with HIP events (render stream) over a second pass
    # of the same K steps right after it; --kernel-events timed puts them inside the timed region.
    in_region = args.kernel_events == "timed"
    rend.kernel_profile(in_region)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter()
    if world > 1 or args.force_dist:
        if trace_host is not None:
            print("host ms/step:", {k: round(v / args.steps * 1e3, 4) for k, v in trace_host.items()}, file=sys.stderr)
    sync()
    t1 = time.perf_counter()
    if not in_region:
        rend.kernel_profile(True)
        for _ in range(args.steps):
            step()
        sync()
    ktimes = rend.kernel_times()
    rend.kernel_profile(False)
    stats = rend.last_stats()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples_per_frame = W * H * aa * aa
    frames_per_step = world if not tiles else 1  # frames mode: every rank renders a whole frame per step
    value = frames_per_step * samples_per_frame * args.steps / elapsed / 1e6

    # roofline of the dominant kernel (rank 0's measurements)
    ktimes = {k: v for k, v in ktimes.items() if v[1]}
    if not ktimes:
        ktimes = {"none": (0.0, 1)}
    dom = max(ktimes, key=lambda k: ktimes[k][0])
    dom_ms, dom_n = ktimes[dom]
    # f64 flops this kernel executed in the last step: the exact leaf tests its walks ran after culling
    # (trace / n1n2 walks; the shade kernel runs the is_shadowed walks) + the shade-event model
    if dom == "trace":
        flops = stats["exact_flops"][0]
    elif dom == "n1n2":
        flops = stats["exact_flops"][2]
    elif dom == "shade":
        flops = stats["exact_flops"][1] + stats["shade_events"] * FLOPS["shade"]
    elif dom == "trace_shade":  # fused: closest-hit walk + shading + shadow walks
        flops = stats["exact_flops"][0] + stats["exact_flops"][1] + stats["shade_events"] * FLOPS["shade"]
    else:
        flops = 0
    launches_per_frame = dom_n / args.steps
    # flops of one step / (this kernel's time per step) == per-launch flops / average launch duration
    achieved = flops / (dom_ms / args.steps / 1e3) / 1e12 if dom_ms > 0 else 0.0
    traffic = None
    entry = {}
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc):
        try:
            per_kernel = json.load(open(pmc))
            # the fused trace+shade launch is the shade_kernel<..., FUSED> instantiation in rocprof's naming
            entry = per_kernel.get(dom) or (per_kernel.get("shade") if dom == "trace_shade" else None) or {}
            traffic = entry.get("hbm_bytes_per_launch")
        except Exception:
            traffic, entry = None, {}
    # SURVEY §8(d) full-scan model for the same rays: what the reference's algorithm would execute
    per_ray = (FLOPS["sphere"] * counts["sphere"] + FLOPS["plane"] * counts["plane"] + FLOPS["group"] * counts["group"]
               + FLOPS["tri"] * counts["tri"])
    if dom == "trace":
        ref_flops = stats["rays"] * per_ray
    elif dom == "n1n2":
        ref_flops = stats["n1n2_scans"] * per_ray
    elif dom == "shade":
        ref_flops = stats["shadow_rays"] * per_ray + stats["shade_events"] * FLOPS["shade"]
    elif dom == "trace_shade":
        ref_flops = (stats["rays"] + stats["shadow_rays"]) * per_ray + stats["shade_events"] * FLOPS["shade"]
    else:
        ref_flops = 0
    ref_tf = ref_flops / (dom_ms / args.steps / 1e3) / 1e12 if dom_ms > 0 else 0.0
    roofline = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP64_PEAK_TFLOPS, 4), "traffic": traffic, "kernel": dom,
                "kernel_ms": round(dom_ms / dom_n, 4),
                "kernel_timing": "HIP events around every launch on the render stream, "
                                 + ("inside the timed region" if in_region else
                                    f"over a second pass of the same {args.steps} steps after the timed region"), "launches_per_step": launches_per_frame,
                "flops_per_launch": flops / launches_per_frame,
                "reference_equivalent": {"tflops": round(ref_tf, 2), "frac": round(ref_tf / FP64_PEAK_TFLOPS, 3),
                                         "flops_per_step": ref_flops,
                                         "model": "SURVEY §8(d) full scan (every ray tests every primitive; "
                                                  "triangles counted as if their group box were hit)"},
                "valu_busy": {"frac": entry.get("valu_busy_frac"), "rocprof_kernel_ms":
                              (entry["rocprof_avg_ns"] / 1e6 if entry.get("rocprof_avg_ns") else None),
                              "source": entry.get("profile"),
                              "model": "SQ_ACTIVE_INST_VALU (quad-cycles) x SQ_WAVES x 4 / (1024 SIMDs x 2.4 GHz x "
                                       "rocprof mean launch time): the share of all SIMD cycles issuing vector "
                                       "instructions, the bound this f64 kernel actually runs into"},
                "note": "achieved = f64 flops the kernel executed: exact leaf tests after culling (SURVEY §8d model: "
                        "sphere 57, plane 13, triangle/group 45) + 250 per shade event for the shade kernel, / kernel "
                        "time; the f32 bundle/line culling that removes the other tests is overhead, not counted. Peak = MI355X FP64 vector = FP64 MFMA "
                        "dense 78.6 TF; bit-parity forbids FMA contraction (DESIGN.md §4)"}

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        from oracle.scene_yaml import build_from_yaml

        threads = min(16, os.cpu_count() or 1)
        o, ocam = build_from_yaml(text, W, H, aa, obj_root=os.path.join(ROOT, "scenes"))
        tc = time.perf_counter()
        canvas, _ = o.render(ocam, max_depth=depth, threads=threads, band=block * aa, band_stride=args.cpu_stride)
        dt = time.perf_counter() - tc
        sel = np.array([y for y in range(H * aa) if (y // (block * aa)) % args.cpu_stride == 0])
        cpu_samples = len(sel) * W * aa
        cpu = {"value": round(cpu_samples / dt / 1e6, 5), "unit": "Mpixel-samples/s", "cores": threads, "kind": "port",
               "sample": f"oracle (C++ restatement, reference structure: per-object inverse, full xs list + stable "
                         f"sort, recursion) on {len(sel) // aa} of {H} output rows (one {block}-row band in every "
                         f"{args.cpu_stride}), {cpu_samples} samples, {dt:.1f}s"}
        avg = o.aa_average(np.nan_to_num(canvas), aa)
        out_rows = sorted(set(int(y) // aa for y in sel))
        gpu_img = tile.cpu().numpy() if not multi else pipe.frame.double().cpu().numpy()
        parity = {"rows_checked": len(out_rows),
                  "max_abs_diff": float(np.max(np.abs(gpu_img[out_rows] - avg[out_rows]))),
                  "bit_exact_frac": float(np.mean(gpu_img[out_rows] == avg[out_rows]))}

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "Mpixel-samples/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "higher_is_better": True,
                "scaling": "strong" if tiles else "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic (scenes/make_scenes.py, seeded)",
                "config": {"workload": args.workload, "scene": scene_file, "width": W, "height": H, "aa": aa,
                           "max_depth": depth, "samples_per_step": samples_per_frame, "objects": counts["objects"],
                           "frames_per_step": frames_per_step,
                           "parallelism": (f"row-tiles x{world}" + (" + pipelined rccl gather (f32 tiles)"
                                                                    if world > 1 else "")) if tiles else
                           f"frame-parallel x{world} (one whole frame per rank per step, no data-path collective)"},
                "roofline": roofline, "cpu_baseline": cpu, "parity_sample": parity,
                "kernels_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in ktimes.items() if v[1]},
                "host_enqueue_ms_per_step": round((t_enq - t0) / args.steps * 1e3, 4),
                "stats_last_step": {k: stats[k] for k in ("rays", "shadow_rays", "shade_events", "n1n2_scans",
                                                          "prim_tests", "exact_flops", "wave_visits")}}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    rend.close()


if __name__ == "__main__":
    main()

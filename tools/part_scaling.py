"""Strong-scaling predictor on one GPU: the C3 frame split into N row-tile parts
(the partition bench.py --gpus N uses), each part rendered alone on this GPU, K frames timed with HIP
events on the render stream.  The slowest part's time is what one rank of an N-GPU run spends per
frame before the transfer, so 1-part time / max part time bounds the N-GPU speedup from above (the
transfer of the runs to rank 0 comes on top, overlapped with the next frame's render).  Each part renders
in one render context here.  Also the virtual group (rr_create_virtual: the N parts, their tiles, the
device-local stand-in for the RCCL transfer) per frame, all parts on this one GPU.
Usage: python tools/part_scaling.py [workload] [steps] [part P N]   ->  JSON on stdout.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import rray_amd as R

    wl = sys.argv[1] if len(sys.argv) > 1 else bench.MULTI_GPU_WORKLOAD
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    scene_file, W, H, aa, depth = bench.WORKLOADS[wl]
    text = open(os.path.join(ROOT, "scenes", scene_file)).read()
    scene = R.YamlScene(text, W, H, aa, obj_root=bench.scene_dir(scene_file))
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    rend = R.Renderer(0)
    rend.upload(scene)
    flags = R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING

    def time_part(part, nparts):
        rows = R.part_rows(H, part, nparts, bench.BLOCK)
        if len(rows) == 0:
            return 0.0
        out = torch.empty((len(rows), W, 3), dtype=torch.float64, device=dev)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, part, nparts, bench.BLOCK, flags)
        for _ in range(2):
            rend.render_device(scene.camera, opts, None, out.data_ptr(), st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            rend.render_device(scene.camera, opts, None, out.data_ptr(), st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / steps

    def time_part_pipelined(part, nparts, k=2):
        """Consecutive frames alternate over k contexts on k streams (frame f on context f % k): one
        frame's latency-bound deep levels overlap the next frame's level 0."""
        rows = R.part_rows(H, part, nparts, bench.BLOCK)
        ctxs = [rend] + [R.Renderer(0) for _ in range(k - 1)]
        for c in ctxs[1:]:
            c.upload(scene)
        sts = [torch.cuda.Stream(dev) for _ in range(k)]
        outs = [torch.empty((len(rows), W, 3), dtype=torch.float64, device=dev) for _ in range(k)]
        opts = R._lib.RenderOpts(aa, depth, 0, 0, part, nparts, bench.BLOCK, flags)
        main = torch.cuda.current_stream(dev)

        def run(nf):
            for f in range(nf):
                j = f % k
                ctxs[j].render_device(scene.camera, opts, None, outs[j].data_ptr(), sts[j].cuda_stream)
        run(2 * k)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for s in sts:
            s.wait_stream(main)
        run(steps * k)
        for s in sts:
            main.wait_stream(s)
        e1.record(main)
        e1.synchronize()
        for c in ctxs[1:]:
            c.close()
        return e0.elapsed_time(e1) / (steps * k)

    res = {"workload": wl, "steps": steps, "parts": {}}
    if len(sys.argv) > 3 and sys.argv[3] == "pipe":  # "pipe": frame-pipelined per-part throughput
        res["pipelined"] = {n: {"part0_ms": round(time_part(0, n), 4), "part0_pipelined_ms": round(time_part_pipelined(0, n), 4)}
                            for n in (1, 8)}
        print(json.dumps(res))
        return
    if len(sys.argv) > 3:  # "part P N": only that part (for a rocprofv3 kernel trace of one rank's levels)
        p, n = int(sys.argv[4]), int(sys.argv[5])
        res["part"] = {"part": p, "nparts": n, "ms": round(time_part(p, n), 4)}
        print(json.dumps(res))
        return
    one = time_part(0, 1)
    res["one_part_ms"] = round(one, 4)
    for n in (2, 4, 8):
        t = [time_part(p, n) for p in range(n)]
        res["parts"][n] = {"part_ms": [round(x, 4) for x in t], "max_part_ms": round(max(t), 4),
                           "sum_parts_ms": round(sum(t), 4), "speedup_bound": round(one / max(t), 3),
                           "balance": round(sum(t) / n / max(t), 4)}
    rend.close()
    for n in (1, 8):  # the whole group path (N parts, padded tiles, local gather stand-in, un-interleave)
        g = R.Renderer.virtual(0, n)
        g.upload(scene)
        frame = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, 0, 1, bench.BLOCK, flags)
        for _ in range(2):
            g.render_gather_device(scene.camera, opts, frame.data_ptr(), st.cuda_stream)
        # the group's renders run on its own streams and wait only for the transfer that last read their tile
        # buffer, not for the caller's stream: drain the warm-up frames first, or the first timed frame's render
        # overlaps them and escapes the events (the round-4 5.16 ms "virtual_group_1" against 6.32 ms per part)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            g.render_gather_device(scene.camera, opts, frame.data_ptr(), st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        res[f"virtual_group_{n}_ms"] = round(e0.elapsed_time(e1) / steps, 4)
        g.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

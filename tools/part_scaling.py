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

    def time_root(nparts, mode):
        """Rank 0's steady state in an nparts-GPU group, emulated on this GPU: its own part rendered on the render stream
        (two tile buffers, the render waiting only for the transfer that last read its buffer, as multi.cpp), and on the
        transfer stream per frame what the root does beyond rendering (mode "stage"): its own tile copied into the
        staging buffer, the other parts' rows written into it (the receives' writes of the incoming bytes: a
        device copy of that many bytes stands in for them) and the placement into frame order (one index_select over
        the stage map, the traffic of multi.cpp's place_tile_kernel).  Mode "render": the render alone."""
        from rray_amd import dist as rdist

        rows = R.part_rows(H, 0, nparts, bench.BLOCK)
        r0 = len(rows)
        tiles = [torch.empty((r0, W, 3), dtype=torch.float64, device=dev) for _ in range(2)]
        stage = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        frame = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        peers = torch.zeros((H - r0, W, 3), dtype=torch.float64, device=dev)
        src = torch.as_tensor(rdist.stage_sources(H, nparts, bench.BLOCK), dtype=torch.long, device=dev)
        s_r, s_c = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        main = torch.cuda.current_stream(dev)
        ev_r = [torch.cuda.Event() for _ in range(2)]
        ev_g = [torch.cuda.Event() for _ in range(2)]
        for e in ev_r + ev_g:
            e.record(main)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, 0, nparts, bench.BLOCK, flags)

        def one(k):
            b = k % 2
            s_r.wait_event(ev_g[b])
            rend.render_device(scene.camera, opts, None, tiles[b].data_ptr(), s_r.cuda_stream)
            ev_r[b].record(s_r)
            if mode == "stage":
                with torch.cuda.stream(s_c):
                    s_c.wait_event(ev_r[b])
                    stage[:r0].copy_(tiles[b])
                    stage[r0:].copy_(peers)
                    torch.index_select(stage, 0, src, out=frame)
            ev_g[b].record(s_c)

        for k in range(4):
            one(k)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        s_r.wait_stream(main)
        s_c.wait_stream(main)
        for k in range(steps):
            one(k)
        main.wait_stream(s_r)
        main.wait_stream(s_c)
        e1.record(main)
        e1.synchronize()
        return e0.elapsed_time(e1) / steps

    def band_opts(y0, y1):
        return R._lib.RenderOpts(aa, depth, 0, 0, 0, 1, bench.BLOCK, flags, y0, y1)

    def time_band(y0, y1):
        if y1 <= y0:
            return 0.0
        out = torch.empty((y1 - y0, W, 3), dtype=torch.float64, device=dev)
        opts = band_opts(y0, y1)
        for _ in range(2):
            rend.render_device(scene.camera, opts, None, out.data_ptr(), st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            rend.render_device(scene.camera, opts, None, out.data_ptr(), st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / steps

    def time_root_band(y0, y1):
        """Rank 0's steady state in the band partition, emulated on this GPU: its band rendered on the render stream
        (two tile buffers), and per frame on the transfer stream its tile copied into the frame's rows and the other
        bands' bytes written into theirs (a device copy of that many bytes stands in for the receives' writes)."""
        r0 = y1 - y0
        tiles = [torch.empty((max(r0, 1), W, 3), dtype=torch.float64, device=dev) for _ in range(2)]
        frame = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        peers = torch.zeros((H - r0, W, 3), dtype=torch.float64, device=dev)
        s_r, s_c = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        main = torch.cuda.current_stream(dev)
        ev_r = [torch.cuda.Event() for _ in range(2)]
        ev_g = [torch.cuda.Event() for _ in range(2)]
        for e in ev_r + ev_g:
            e.record(main)
        opts = band_opts(y0, y1)

        def one(k):
            b = k % 2
            s_r.wait_event(ev_g[b])
            if r0 > 0:
                rend.render_device(scene.camera, opts, None, tiles[b].data_ptr(), s_r.cuda_stream)
            ev_r[b].record(s_r)
            with torch.cuda.stream(s_c):
                s_c.wait_event(ev_r[b])
                if r0 > 0:
                    frame[y0:y1].copy_(tiles[b][:r0])
                frame[:y0].copy_(peers[:y0])
                frame[y1:].copy_(peers[y0:])
            ev_g[b].record(s_c)

        for k in range(4):
            one(k)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        s_r.wait_stream(main)
        s_c.wait_stream(main)
        for k in range(steps):
            one(k)
        main.wait_stream(s_r)
        main.wait_stream(s_c)
        e1.record(main)
        e1.synchronize()
        return e0.elapsed_time(e1) / steps

    def time_group(n, interleave=False, bounds=None):
        g = R.Renderer.virtual(0, n)
        g.upload(scene)
        if bounds is not None:
            g.set_bands(bounds)
        frame = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        opts = R._lib.RenderOpts(aa, depth, 0, 0, 0, 1, bench.BLOCK,
                                 flags | (R._lib.RR_PART_INTERLEAVE if interleave else 0))
        for _ in range(2):
            g.render_gather_device(scene.camera, opts, frame.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            g.render_gather_device(scene.camera, opts, frame.data_ptr(), st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        b = g.bands()
        g.close()
        return e0.elapsed_time(e1) / steps, b

    res = {"workload": wl, "steps": steps, "parts": {}}
    if len(sys.argv) > 3 and sys.argv[3] == "bands":  # the band partition (the library default at N > 1)
        one = time_part(0, 1)
        res["one_part_ms"] = round(one, 4)
        res["bands"] = {}
        for n in (2, 4, 8):
            vg, b = time_group(n)  # calibrates the bands (rank 0's timed bands, rr_balance_bands)
            t = [time_band(b[p], b[p + 1]) for p in range(n)]
            root = time_root_band(b[0], b[1])
            worst = max(t[1:] + [root])
            res["bands"][n] = {"bounds": b, "part_ms": [round(x, 4) for x in t], "root_with_transfer_ms": round(root, 4),
                               "max_part_ms": round(max(t), 4), "sum_parts_ms": round(sum(t), 4),
                               "virtual_group_ms": round(vg, 4),
                               "virtual_group_over_sum_of_parts": round(vg / sum(t), 4),
                               "speedup_bound": round(one / max(t), 3),
                               "speedup_bound_with_root_transfer": round(one / worst, 3)}
        vi, _ = time_group(8, interleave=True)
        res["virtual_group_8_interleave_ms"] = round(vi, 4)
        print(json.dumps(res))
        return
    if len(sys.argv) > 3 and sys.argv[3] == "root":  # "root": rank 0's per-frame time with its transfer work overlapped
        one = time_part(0, 1)
        res["one_part_ms"] = round(one, 4)
        res["root"] = {}
        for n in (2, 4, 8):
            t_parts = [time_part(p, n) for p in range(n)]
            t_render, t_stage = time_root(n, "render"), time_root(n, "stage")
            worst = max(t_parts[1:] + [t_stage])
            res["root"][n] = {"part_ms": [round(x, 4) for x in t_parts], "root_render_pipelined_ms": round(t_render, 4),
                              "root_with_transfer_ms": round(t_stage, 4),
                              "speedup_bound_with_root_transfer": round(one / worst, 3)}
        print(json.dumps(res))
        return
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

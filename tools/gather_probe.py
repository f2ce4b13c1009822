"""Probe: host-side cost of each call in the pipelined gather step at 1 rank (RCCL)."""
import time, torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dev = torch.device("cuda", 0)
H, W = 1080, 1920
tiles = [torch.zeros((H, W, 3), dtype=torch.float32, device=dev) for _ in range(2)]
big = torch.empty((1, H, W, 3), dtype=torch.float32, device=dev)
gl = list(big.unbind(0))
idx = torch.arange(H, device=dev)
fr = torch.empty_like(tiles[0])
rs = torch.cuda.Stream(dev)
pend = [None, None]
acc = {}
def tic(name, t0):
    t = time.perf_counter(); acc[name] = acc.get(name, 0) + (t - t0); return t
for k in range(40):
    if k == 10:
        torch.cuda.synchronize(); acc.clear(); T0 = time.perf_counter()
    t = time.perf_counter()
    i = k % 2
    with torch.cuda.stream(rs):
        if pend[i] is not None:
            pend[i].wait()
        t = tic("prev.wait", t)
        tiles[i].add_(1.0)  # stand-in for the render
        t = tic("render(add_)", t)
    torch.cuda.current_stream(dev).wait_stream(rs)
    t = tic("wait_stream", t)
    w = dist.gather(tiles[i], gather_list=gl, dst=0, async_op=True)
    t = tic("gather(async)", t)
    pend[i] = w
    w.wait()
    t = tic("work.wait", t)
    torch.index_select(big.view(H, W, 3), 0, idx, out=fr)
    t = tic("index_select", t)
T1 = time.perf_counter()
torch.cuda.synchronize()
print({k: round(v / 30 * 1e3, 4) for k, v in acc.items()}, "host ms/step", round((T1 - T0) / 30 * 1e3, 4), flush=True)
dist.destroy_process_group()

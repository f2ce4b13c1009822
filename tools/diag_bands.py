import json, os, sys
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench, rray_amd as R
wl = "c3_s1024_reflect"
scene_file, W, H, aa, depth = bench.WORKLOADS[wl]
text = open(os.path.join("scenes", scene_file)).read()
scene = R.YamlScene(text, W, H, aa, obj_root=bench.scene_dir(scene_file))
dev = torch.device("cuda", 0); st = torch.cuda.Stream(dev)
rend = R.Renderer(0); rend.upload(scene)
flags = R._lib.RR_OUT_AVG | R._lib.RR_NO_FRAME_TIMING
def tb(y0, y1, steps=3):
    out = torch.empty((y1 - y0, W, 3), dtype=torch.float64, device=dev)
    o = R._lib.RenderOpts(aa, depth, 0, 0, 0, 1, 8, flags, y0, y1)
    for _ in range(2): rend.render_device(scene.camera, o, None, out.data_ptr(), st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps): rend.render_device(scene.camera, o, None, out.data_ptr(), st.cuda_stream)
    e1.record(st); e1.synchronize()
    return e0.elapsed_time(e1) / steps
res = {}
for hb in (40, 120, 270):
    bands = [(y, min(H, y + hb)) for y in range(0, H, hb)]
    t = [tb(a, b) for a, b in bands]
    res[hb] = {"times": [round(x, 4) for x in t], "sum": round(sum(t), 4)}
res["full"] = tb(0, H)
res["b0_552"] = tb(0, 552)
res["b_1048_1256"] = tb(1048, 1256)
print(json.dumps(res))

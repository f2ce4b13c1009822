"""Probe: the reference's examples/area_light.png (one random thread_rng draw) against GPU renders of
the same scene under several jitter seeds, per candidate aa.  Pixels whose quantised value is the same
under every seed do not depend on the jitter and must match the reference exactly; the rest
(penumbra) are compared statistically."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rray_amd as R  # noqa: E402
from PIL import Image  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
text = open(os.path.join(ROOT, "scenes", "c5_area_light.yaml")).read()
ref = np.asarray(Image.open(os.path.join(GOLDEN, "png", "area_light.png")).convert("RGB")).astype(np.int32)
r = R.Renderer(0)
for aa in [int(a) for a in os.environ.get("AAS", "1,2,3").split(",")]:
    scene = R.YamlScene(text, 800, 400, aa, obj_root=GOLDEN)
    r.upload(scene)
    qs = [R.quantize(r.render(scene.camera, aa=aa, seed=s)["avg"])[..., :3].astype(np.int32) for s in range(8)]
    Q = np.stack(qs)
    stable = (Q == Q[0]).all(axis=0).all(axis=2)
    st_diff = int(((Q[0] != ref).any(axis=2) & stable).sum())
    pen = ~stable
    lo, hi = Q.min(axis=0), Q.max(axis=0)
    inside = ((ref >= lo - 2) & (ref <= hi + 2)).all(axis=2)
    mean = Q.mean(axis=0)
    print(f"aa={aa}: stable {int(stable.sum())} px, of which differ from the reference {st_diff}; penumbra "
          f"{int(pen.sum())} px: ref within seed range+-2 {float(inside[pen].mean()) if pen.any() else 1:.4f}, "
          f"mean |ref - mean| {float(np.abs(ref - mean)[pen].mean()) if pen.any() else 0:.3f}, "
          f"max {float(np.abs(ref - mean)[pen].max()) if pen.any() else 0:.1f}", flush=True)
    d = np.abs(Q[0] - ref).max(axis=2)
    sd = d[stable]
    print("   stable |diff| histogram:", {k: int((sd == k).sum()) for k in range(0, 6)}, ">5:", int((sd > 5).sum()))
    ys, xs = np.nonzero((d > 0) & stable)
    if len(ys):
        print("   differing stable rows", np.percentile(ys, [0, 25, 50, 75, 100]), "cols", np.percentile(xs, [0, 25, 50, 75, 100]))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"area_aa{aa}.npz"), q=Q.astype(np.uint8), stable=stable)

"""Probe (CPU, this container only: reads /root/reference): the pinned oracle renders the reference's
examples/objects/torus.yaml (PIL decodes its JPEG texture) and compares with examples/objects/torus.png."""
import os, sys, time, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.scene_yaml import build_from_yaml
from PIL import Image
ref_dir = '/root/reference'
text = open(os.path.join(ref_dir, 'examples/objects/torus.yaml')).read()
ref = np.asarray(Image.open(os.path.join(ref_dir, 'examples/objects/torus.png')).convert('RGB'))
for aa in (3,):
    t = time.time()
    o, cam = build_from_yaml(text, 800, 400, aa, obj_root=ref_dir)
    canvas, st = o.render(cam, max_depth=5, threads=8)
    q = o.quantize(o.aa_average(canvas, aa))[..., :3]
    d = np.abs(q.astype(int) - ref.astype(int)).max(axis=2)
    print(aa, 'time', round(time.time() - t, 1), 'differ', int((d > 0).sum()), 'max', int(d.max()), 'hist', {k: int((d == k).sum()) for k in range(1, 5)}, flush=True)
    np.save('/tmp/torus_oracle_q.npy', q)

"""Regenerates tests/golden/oracle_*.npy: AA-averaged f64 images rendered by the CPU oracle
(oracle/rray_oracle.cpp, pinned by the reference's known-answer tests) for small versions of the
BASELINE config scenes.  The GPU tests compare the HIP path against these committed vectors.
Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.scene_yaml import build_from_yaml  # noqa: E402

CASES = [("c1_readme.yaml", 40, 30, 2, 0), ("c2_s1024.yaml", 48, 27, 1, 0), ("c3_s1024_reflect.yaml", 32, 18, 2, 0),
         ("c4_teapot.yaml", 32, 18, 1, 0), ("c5_area_light.yaml", 32, 16, 2, 3),
         # each config at its own AA level (BASELINE configs: C3 aa=3, C4 aa=2)
         ("c3_s1024_reflect.yaml", 32, 18, 3, 0), ("c4_teapot.yaml", 32, 18, 2, 0)]


def main():
    meta = []
    for scene, W, H, aa, seed in CASES:
        text = open(os.path.join(ROOT, "scenes", scene)).read()
        o, cam = build_from_yaml(text, W, H, aa, obj_root=os.path.join(ROOT, "scenes"))
        canvas, st = o.render(cam, max_depth=5, seed=seed)
        avg = o.aa_average(canvas, aa)
        name = f"oracle_{scene[:-5]}_{W}x{H}_aa{aa}.npy"
        np.save(os.path.join(HERE, name), avg)
        meta.append({"scene": scene, "W": W, "H": H, "aa": aa, "seed": seed, "file": name, "stats": st})
        print(name, st)
    json.dump(meta, open(os.path.join(HERE, "golden_renders.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

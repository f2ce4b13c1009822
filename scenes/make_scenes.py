"""Writes the BASELINE.json workload scenes as rray YAML files.

  c1_readme.yaml          README.md:56-103 scene (1 glass/reflective sphere + checker plane)
  c2_s1024.yaml           synthetic 32x32 sphere grid + checker plane, point light
  c3_s1024_reflect.yaml   same, spheres with (i+j)%4==0 reflective 0.5, plane reflective 0.3
  c4_teapot.yaml          teapot.obj (6320 smooth triangles) + checker plane (example1.yaml teapot xform)
  c5_area_light.yaml      examples/area_light.yaml, copied verbatim (bare-CR line endings)

Colours are rounded to 3 decimals so the YAML text round-trips exactly through both front-ends.
Run: python scenes/make_scenes.py   (outputs are committed)
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

HEADER = """camera:
  fov: 60
  from: [0, 6, -6]
  to: [0, 0, 8]
  up: [0, 1, 0]
lights:
  - type: point
    color: [1, 1, 1]
    position: [-10, 10, -10]
scene:
"""
PLANE = """  - type: plane
    transforms: []
    material:
      pattern:
        type: checker
        pattern_a:
          type: solid
          color: [0.25, 0.25, 0.75]
          transforms: []
        pattern_b:
          type: solid
          color: [0.75, 0.75, 0.75]
          transforms: []
        transforms:
          - type: scale
            amount: [1, 1, 1]
      ambient: 0.1
      diffuse: 0.9
      specular: 0
      shininess: 200
      reflective: {refl}
"""
SPHERE = """  - type: sphere
    transforms:
      - type: scale
        amount: [0.2, 0.2, 0.2]
      - type: translate
        amount: [{x}, 0.25, {z}]
    material:
      pattern:
        type: solid
        color: [{r}, {g}, {b}]
      ambient: 0.1
      diffuse: 0.9
      specular: 0.9
      shininess: 200
      reflective: {refl}
"""


def fmt(v):
    s = repr(float(v))
    return s


def s1024(reflective):
    rng = np.random.default_rng(20241015)
    cols = np.round(rng.uniform(0.1, 1.0, (1024, 3)), 3)
    out = [HEADER, PLANE.format(refl="0.3" if reflective else "0")]
    k = 0
    for i in range(32):
        for j in range(32):
            x = (i - 15.5) * 0.5
            z = (j - 15.5) * 0.5 + 8
            refl = "0.5" if (reflective and (i + j) % 4 == 0) else "0"
            r, g, b = (("%.3f" % c) for c in cols[k])
            out.append(SPHERE.format(x=fmt(x), z=fmt(z), r=r, g=g, b=b, refl=refl))
            k += 1
    return "".join(out)


README = """camera:
  fov: 60
  from: [0, 2.5, -5.0]
  to: [0,1,0]
  up: [0,1,0]
lights:
  - type: point
    color: [1,1,1]
    position: [-10,10,-10]
scene:
  - type: plane
    transforms: []
    material:
      pattern:
        type: checker
        pattern_a:
          type: solid
          color: [0.25, 0.25, 0.75]
          transforms: []
        pattern_b:
          type: solid
          color: [0.75, 0.75, 0.75]
          transforms: []
        transforms:
          - type: scale
            amount: [1, 1, 1]
      ambient: 0.1
      diffuse: 0.9
      specular: 0
      shininess: 200
  - type: sphere
    transforms:
     - type: translate
       amount: [0, 1, 2]
     - type: scale
       amount: [0.5, 0.5, 0.5]
    material:
     pattern:
       type: solid
       color: [1, 0, 0]
       transforms: []
     ambient: 0.1
     diffuse: 0.9
     specular: 0.9
     shininess: 200
     reflective: 0.9
     transparency: 0.1
     refractive_index: 1.5
"""

TEAPOT = """camera:
  fov: 60
  from: [0, 1.5, -5.0]
  to: [0,1,0]
  up: [0,1,0]
lights:
  - type: point
    color: [1,1,1]
    position: [-10,10,-10]
scene:
""" + PLANE.format(refl="0") + """  - type: obj_file
    obj_file: teapot.obj
    material:
      pattern:
        type: solid
        color: [0.302, 0.71, 0.98]
      ambient: 0.1
      diffuse: 0.7
      specular: 0.9
      shininess: 300
      reflective: 0
      transparency: 0
      refractive_index: 1.52
    transforms:
      - type: rotate
        axis: x
        angle: -90
      - type: rotate
        axis: 'y'
        angle: 130
      - type: scale
        amount: [0.05, 0.05, 0.05]
      - type: translate
        amount: [-1.75, 0, 0]
"""


def main():
    files = {"c1_readme.yaml": README, "c2_s1024.yaml": s1024(False), "c3_s1024_reflect.yaml": s1024(True),
             "c4_teapot.yaml": TEAPOT}
    for name, text in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            f.write(text)
    print("wrote", ", ".join(files))


if __name__ == "__main__":
    main()

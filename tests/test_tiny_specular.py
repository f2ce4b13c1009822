"""The tiny-specular skip of light_terms (device_core.inc), checked on the CPU.

A lit lane skips the specular pow when, in f32, shininess * log2(reflect.eye) <= -71 (reflect.eye >= 2^-100,
shininess <= 1e4) and (|Ix| + |Iy| + |Iz|) |specular| 2^-15 < |diffuse_c| for every channel.  The claim: for such a
lane the reference's diffuse + (I * specular) * powf(reflect.eye, shininess) (light.rs:133,138) equals diffuse
bit for bit.  Here the condition is restated with numpy's f32 log2 and the sum is evaluated with Python floats
(IEEE doubles, libm pow) on inputs drawn at and around the thresholds.
"""
import math

import numpy as np


def tiny(rde, shininess, intensity, specular, diffuse):
    """The kernel's condition (light_terms<true>), NaN-safe in the same way."""
    rf = np.float32(rde)
    if not (rf >= np.float32(2.0 ** -100) and shininess <= 1e4):
        return False
    with np.errstate(all="ignore"):
        lg = np.float32(shininess) * np.log2(rf)
    if not (lg <= np.float32(-71.0)):
        return False
    dlim = (abs(intensity[0]) + abs(intensity[1]) + abs(intensity[2])) * abs(specular) * 2.0 ** -15
    return all(dlim < abs(d) for d in diffuse)


def reference_dspec(rde, shininess, intensity, specular, diffuse):
    factor = math.pow(rde, shininess)
    return [d + (i * specular) * factor for d, i in zip(diffuse, intensity)]


def test_skipped_lanes_keep_diffuse_exactly():
    rng = np.random.default_rng(20261018)
    checked = 0
    for _ in range(100_000):
        shininess = float(rng.choice([1.0, 10.0, 50.0, 200.0, 300.0, 1000.0, 1e4, rng.uniform(0.5, 1e4)]))
        # reflect.eye near the threshold 2^(-71 / shininess), on both sides
        thr = 2.0 ** (-71.0 / shininess)
        rde = float(min(1.0, thr * (1.0 + rng.uniform(-0.02, 0.002))))
        intensity = [float(x) for x in rng.choice([1.0, rng.uniform(0, 4)], size=3)]
        specular = float(rng.uniform(0, 2))
        scale = (abs(intensity[0]) + abs(intensity[1]) + abs(intensity[2])) * specular * 2.0 ** -15
        # diffuse channels just above the bound, or anywhere up to O(1)
        diffuse = [float(scale * (1.0 + rng.uniform(0, 1e-3)) if rng.random() < 0.5 else rng.uniform(0, 1)) for _ in range(3)]
        if not tiny(rde, shininess, intensity, specular, diffuse):
            continue
        checked += 1
        assert reference_dspec(rde, shininess, intensity, specular, diffuse) == diffuse, (rde, shininess, intensity,
                                                                                          specular, diffuse)
    assert checked > 5_000


def test_condition_refuses_nan_and_extremes():
    inten = [1.0, 1.0, 1.0]
    assert not tiny(float("nan"), 200.0, inten, 0.9, [0.5, 0.5, 0.5])
    assert not tiny(0.5, float("nan"), inten, 0.9, [0.5, 0.5, 0.5])
    assert not tiny(0.5, 200.0, [float("nan"), 1.0, 1.0], 0.9, [0.5, 0.5, 0.5])
    assert not tiny(0.5, 200.0, inten, float("inf"), [0.5, 0.5, 0.5])
    assert not tiny(0.5, 200.0, inten, 0.9, [0.5, float("nan"), 0.5])
    assert not tiny(0.5, 200.0, inten, 0.9, [0.5, 0.0, 0.5])  # a zero diffuse channel keeps the pow
    assert not tiny(2.0 ** -120, 0.001, inten, 0.9, [0.5, 0.5, 0.5])  # f32 underflow of reflect.eye
    assert not tiny(0.5, 2e4, inten, 0.9, [0.5, 0.5, 0.5])  # shininess beyond the f32 error budget
    assert not tiny(0.9, 200.0, inten, 0.9, [0.5, 0.5, 0.5])  # the highlight: 0.9^200 = 2^-30.4
    assert tiny(0.5, 200.0, inten, 0.9, [0.5, 0.5, 0.5])

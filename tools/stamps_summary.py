"""Summarise an RR_STAMPS dump (abtest/stamps, $RRAY_STAMPS; tools/stamps_run.sh) of the fused level-0 shade kernel:
mean s_memtime cycles per wave between phase marks.  Region 1 = shade kernel marks, region 0 =
the shadow walk and extra marks (render.hip, RR_STAMPX)."""
import sys

import numpy as np


def main(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(2, 1 << 16, 16).astype(np.int64)
    r0, r1 = a[0], a[1]
    ok = (r1[:, 0] > 0) & (r1[:, 7] > 0)
    r0, r1 = r0[ok], r1[ok]
    hit = r0[:, 0] > 0  # waves with at least one hit (prepare ran)
    rows = [("camera ray + trace prelude", r1[:, 2] - r1[:, 0], ok[ok]),
            ("trace bundle", r1[:, 3] - r1[:, 2], ok[ok]),
            ("trace walk", r1[:, 4] - r1[:, 3], ok[ok]),
            ("-> prepare", r0[:, 5] - r1[:, 4], hit),
            ("prepare", r0[:, 0] - r0[:, 5], hit),
            ("schlick / children", r1[:, 1] - r0[:, 0], hit),
            ("queue appends", r1[:, 5] - r1[:, 1], ok[ok]),
            ("pattern", r0[:, 1] - r1[:, 5], hit),
            ("prelit + shadow prelude", r0[:, 2] - r0[:, 1], hit),
            ("shadow bundle", r0[:, 3] - r0[:, 2], hit),
            ("shadow walk", r0[:, 4] - r0[:, 3], hit),
            ("light final", r1[:, 6] - r0[:, 4], hit),
            ("deliver + flush", r1[:, 7] - r1[:, 6], ok[ok]),
            ("total", r1[:, 7] - r1[:, 0], ok[ok])]
    print(f"waves: {ok.sum()}  with hits: {hit.sum()}")
    for name, d, m in rows:
        d = d[m]
        d = d[(d >= 0) & (d < 1e8)]
        print(f"{name:28s} mean {d.mean():9.0f}  median {np.median(d):9.0f}  (n={d.size})")
    for name, r in (("trace walk", r1), ("shadow walk", r0)):
        w = np.maximum(r[:, 11], 1)
        print(f"{name}: per walk  bundle-candidate chunks {np.mean(r[:, 8] / w):.2f}  "
              f"line-passing chunks {np.mean(r[:, 9] / w):.2f}  candidate nodes {np.mean(r[:, 10] / w):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])


def occupancy(path):
    """Kernel-entry stamps (slot 12) and hardware ids (13: HW_ID, 14: XCC_ID): time before phase 0
    (counter clear + cull staging) and how fully each CU's 16 wave slots were kept busy."""
    a = np.fromfile(path, dtype=np.uint64).reshape(2, 1 << 16, 16).astype(np.int64)
    r1 = a[1]
    ok = (r1[:, 12] > 0) & (r1[:, 7] > 0)
    r1 = r1[ok]
    if not len(r1):
        return
    ent, end, p0 = r1[:, 12], r1[:, 7], r1[:, 0]
    print(f"entry -> phase 0 (clear + staging): mean {np.mean(p0 - ent):.0f}  median {np.median(p0 - ent):.0f}")
    hw, xcc = r1[:, 13], r1[:, 14] & 0xf
    cu = (xcc << 8) | (((hw >> 13) & 0x7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf)
    simd = (cu << 2) | ((hw >> 4) & 3)
    effs, spans = [], []
    for c in np.unique(cu):
        m = cu == c
        span = end[m].max() - ent[m].min()
        spans.append(span)
        effs.append(np.sum(end[m] - ent[m]) / (span * 16.0))
    print(f"CUs {len(effs)}  span mean {np.mean(spans):.0f} min {np.min(spans):.0f} max {np.max(spans):.0f}  "
          f"wave-slot occupancy mean {np.mean(effs):.3f}")
    per_simd = np.bincount(np.searchsorted(np.unique(simd), simd))
    print(f"waves per SIMD: mean {per_simd.mean():.1f} min {per_simd.min()} max {per_simd.max()}")
    print(f"wave life (entry -> end): mean {np.mean(end - ent):.0f}")


if __name__ == "__main__" and len(sys.argv) > 1:
    occupancy(sys.argv[1])

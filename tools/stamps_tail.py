"""Tail analysis of an RR_STAMPS dump: percentiles of per-wave cycles and of the shadow / trace walks'
bundle-candidate nodes, and the share of all wave cycles spent in the slowest 1 % of waves."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(2, 1 << 16, 16).astype(np.int64)
r0, r1 = a[0], a[1]
ok = (r1[:, 0] > 0) & (r1[:, 7] > 0)
hit = ok & (r0[:, 0] > 0)
tot = (r1[:, 7] - r1[:, 0])[ok]
print("wave cycles p50/p90/p99/p99.9/max", np.percentile(tot, [50, 90, 99, 99.9, 100]).astype(int))
srt = np.sort(tot)
print("share of cycles in the slowest 1 % of waves", round(float(srt[int(0.99 * len(srt)):].sum() / srt.sum()), 3))
for name, r, m in (("trace", r1, ok), ("shadow", r0, hit)):
    w = np.maximum(r[:, 11][m], 1)
    print(f"{name} walk cycles p50/p99/max", np.percentile((r[:, 4] - r[:, 3])[m], [50, 99, 100]).astype(int),
          " candidate nodes/walk p50/p99/max", np.percentile(r[:, 10][m] / w, [50, 99, 100]))

"""Median duration and gap of consecutive launches per kernel name in a rocprofv3 kernel-trace CSV."""
import csv
import statistics as S
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for a, b in zip(rows, rows[1:]):
    if a["Kernel_Name"] == b["Kernel_Name"]:
        by.setdefault(a["Kernel_Name"], []).append(((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3,
                                                     (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3))
for k, v in by.items():
    print(f"{k[:40]:40s} n={len(v)} duration {S.median(d for d, _ in v):8.2f} us  gap {S.median(g for _, g in v):6.2f} us")

"""Per-level breakdown of a rocprofv3 session (tools/profile_session.sh output dir): for every rr:: kernel
variant and its position inside a frame (level), the mean duration (kernel trace) and the per-dispatch
PMC counters (SQ_WAVES, SQ_INSTS_VALU, ... from the pmc_* passes), matched by dispatch order.
Usage: python tools/profile_levels.py gpurun_out/prof [out.json]
"""
import collections
import csv
import json
import os
import re
import sys


def short(name):
    m = re.search(r"rr::(\w+)<([^>]*)>", name) or re.search(r"rr::(\w+)", name)
    if not m:
        return None
    return m.group(1) + (f"<{m.group(2)}>" if m.lastindex and m.lastindex >= 2 else "")


def frames(rows, key):
    """Label each rr:: dispatch with (short name, occurrence index inside its frame).  A frame starts at
    each dispatch of the first rr:: kernel seen other than the kernels that run once per camera or layout (the
    camera bundles, the first frame's tile-order guess) or every few frames (the tile-order sort)."""
    occasional = {"tile_bundle_kernel", "pixel_wave_bundle_kernel", "tile_guess_kernel", "tile_hist_kernel",
                  "tile_scan_kernel", "tile_scatter_kernel"}
    out, first, seen = [], None, collections.Counter()
    for r in rows:
        k = short(r["Kernel_Name"])
        if not k:
            continue
        if first is None and k not in occasional:  # once per camera / layout, not per frame
            first = k
        if k == first:
            seen = collections.Counter()
        out.append(((k, seen[k]), r))
        seen[k] += 1
    return out


def main(src, out_json=None):
    trace = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))))
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))
    dur = collections.defaultdict(list)
    for key, r in frames(trace, "Kernel_Name"):
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)  # us
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc") or not os.path.exists(f):
            continue
        per_disp = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            d = per_disp.setdefault(int(r["Dispatch_Id"]), {"Kernel_Name": r["Kernel_Name"], "c": collections.Counter()})
            d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        rows = [dict(Kernel_Name=v["Kernel_Name"], c=v["c"]) for _, v in sorted(per_disp.items())]
        for key, r in frames(rows, "Kernel_Name"):
            for c, v in r["c"].items():
                pmc[key][c].append(v)
    res = []
    for key in sorted(dur, key=lambda k: (k[1], k[0])):
        d = dur[key]
        row = {"kernel": key[0], "pos": key[1], "calls": len(d), "mean_us": sum(d) / len(d)}
        for c, v in pmc.get(key, {}).items():
            row[c] = sum(v) / len(v)
        if row.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY"):
                if c in row:
                    row[c + "_per_wave"] = row[c] / row["SQ_WAVES"]
            if "SQ_ACTIVE_INST_VALU" in row:  # quad-cycles summed over waves / all SIMD cycles of the launch
                row["valu_busy"] = 4.0 * row["SQ_ACTIVE_INST_VALU"] / (1024 * 2.4e9 * row["mean_us"] * 1e-6)
        res.append(row)
        print(f"{key[0]:52s} pos {key[1]:2d} x{len(d):4d} {row['mean_us']:9.1f} us  waves {row.get('SQ_WAVES', 0):9.0f}  "
              f"valu/wave {row.get('SQ_INSTS_VALU_per_wave', 0):7.0f}  busy {row.get('valu_busy', 0):.2f}  "
              f"HBM {((2 * row.get('FETCH_SIZE', 0) + row.get('WRITE_SIZE', 0)) * 1024 / 1e6):8.1f} MB")
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])

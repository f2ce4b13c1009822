"""Summarize a rocprofv3 session (tools/profile_session.sh) into profiles/<tag>_summary.json + copies.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reads exactly half of a wide coalesced stream's bytes, so it is doubled.
"""
import collections
import csv
import json
import os
import shutil
import sys


N_SIMDS = 256 * 4    # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
CLOCK_HZ = 2.4e9     # max clock


def per_kernel(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in agg.items()}


def short(name):
    for key in ("trace_kernel", "shadow_kernel", "shade_kernel", "finish_kernel", "combine_kernel", "aa_kernel",
                "n1n2_kernel"):
        if key in name:
            return key.replace("_kernel", "")
    return None


def main(src, tag, workload="c2_s1024"):
    os.makedirs("profiles", exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))))
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    sq = per_kernel(os.path.join(src, "pmc_sq", "run_counter_collection.csv"))
    sq2_path = os.path.join(src, "pmc_sq2", "run_counter_collection.csv")
    sq2 = per_kernel(sq2_path) if os.path.exists(sq2_path) else {}
    out = {"workload": workload, "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE | WRITE_SIZE | "
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES (separate passes)", "kernels": {}}
    for r in stats:
        k = short(r["Name"])
        if not k:
            continue
        f = fetch.get(r["Name"], {}).get("FETCH_SIZE")
        w = write.get(r["Name"], {}).get("WRITE_SIZE")
        s = dict(sq2.get(r["Name"], {}))
        s.update(sq.get(r["Name"], {}))
        hbm = None if f is None or w is None else (2 * f + w) * 1024
        out["kernels"][k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                             "pct": float(r["Percentage"]), "fetch_kib_raw": f, "write_kib": w,
                             "hbm_bytes_per_launch": hbm,
                             "valu_insts_per_wave": (s["SQ_INSTS_VALU"] / s["SQ_WAVES"]) if s.get("SQ_WAVES") else None,
                             # per-wave averages of every SQ counter (SQ_WAVE_CYCLES / WAIT / ACTIVE in quad-cycles)
                             "sq_per_wave": {c: v / s["SQ_WAVES"] for c, v in s.items()
                                             if c.startswith("SQ_") and c != "SQ_WAVES"} if s.get("SQ_WAVES") else None,
                             "sq_waves": s.get("SQ_WAVES"), "grbm_gui_active": s.get("GRBM_GUI_ACTIVE")}
        # VALU busy: SQ_ACTIVE_INST_VALU (quad-cycles per wave) summed over the launch's waves, over every
        # SIMD's cycles of the launch (1024 SIMDs at the 2.4 GHz max clock: a lower bound on the fraction)
        if s.get("SQ_WAVES") and s.get("SQ_ACTIVE_INST_VALU"):
            busy = 4.0 * s["SQ_ACTIVE_INST_VALU"] / (N_SIMDS * CLOCK_HZ * float(r["AverageNs"]) * 1e-9)
            out["kernels"][k]["valu_busy_frac"] = busy
    json.dump(out, open(f"profiles/{tag}_summary.json", "w"), indent=1)
    json.dump({k: {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "valu_busy_frac": v.get("valu_busy_frac"),
                   "rocprof_avg_ns": v["avg_ns"], "profile": f"profiles/{tag}_summary.json"}
               for k, v in out["kernels"].items()},
              open(f"profiles/pmc_{workload}.json", "w"), indent=1)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), f"profiles/{tag}_kernel_stats.csv")
    for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        if os.path.exists(os.path.join(src, p, "run_counter_collection.csv")):
            shutil.copy(os.path.join(src, p, "run_counter_collection.csv"), f"profiles/{tag}_{p}.csv")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))

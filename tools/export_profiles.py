"""Copy a tools/profile_all.sh session into profiles/ (tracked):
  profiles/<tag>/<wl>_levels.json        per kernel variant and level: rocprof mean duration + PMC counters
  profiles/<tag>/<wl>_kernel_stats.csv   rocprofv3 --stats summary
  profiles/<tag>/<wl>_summary.json       the fused trace+shade kernel over a frame (what bench.py's roofline
                                         names "trace_shade"): launches, mean launch, HBM bytes and VALU busy
  profiles/pmc_<wl>.json                 the numbers bench.py attaches to its roofline (traffic, valu_busy)
HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB per MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts half of a
wide coalesced stream).  Usage: python tools/export_profiles.py r02 [workloads...]
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def export(tag, wl):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{wl}")
    levels = json.load(open(os.path.join(src, "levels.json")))
    out_dir = os.path.join(ROOT, "profiles", tag)
    os.makedirs(out_dir, exist_ok=True)
    json.dump(levels, open(os.path.join(out_dir, f"{wl}_levels.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(out_dir, f"{wl}_kernel_stats.csv"))
    # the frame's render kernels: the chain kernel (scenes with reflections: one launch per frame, bench.py's "chain")
    # or the fused trace+shade kernel per level ("trace_shade")
    chain = [r for r in levels if r["kernel"].startswith(("chain_kernel", "tree_kernel"))]
    shade = chain or [r for r in levels if r["kernel"].startswith("shade_kernel")]
    key = "chain" if chain else "trace_shade"
    n = len(shade)  # launches per frame (levels)
    tot_us = sum(r["mean_us"] for r in shade)
    hbm = [(2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024 for r in shade if "FETCH_SIZE" in r and "WRITE_SIZE" in r]
    busy_w = sum(r.get("valu_busy", 0) * r["mean_us"] for r in shade)
    summary = {
        "workload": wl, "kernel": ("chain (chain_kernel / tree_kernel: every reflection chain or color_at tree inside its "
                                   "camera wave, one launch)"
                                   if chain else "trace_shade (shade_kernel<..., FUSED, ...>, one launch per level)"),
        "launches_per_frame": n, "frame_kernel_us": round(tot_us, 2), "mean_launch_us": round(tot_us / n, 2),
        "hbm_bytes_per_launch": (sum(hbm) / len(hbm)) if len(hbm) == n else None,
        "valu_busy": round(busy_w / tot_us, 4) if tot_us else None,
        "levels": [{k: r.get(k) for k in ("kernel", "pos", "mean_us", "SQ_WAVES", "SQ_INSTS_VALU_per_wave",
                                             "valu_busy", "FETCH_SIZE", "WRITE_SIZE")} for r in shade],
        "others": [{k: r.get(k) for k in ("kernel", "pos", "mean_us", "FETCH_SIZE", "WRITE_SIZE")}
                   for r in levels if r not in shade],
        "source": "rocprofv3 --kernel-trace --stats; separate --pmc passes (SQ_WAVES SQ_INSTS_VALU "
                  "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
                  "SQ_INSTS_SALU | FETCH_SIZE | WRITE_SIZE), tools/profile_all.sh",
    }
    json.dump(summary, open(os.path.join(out_dir, f"{wl}_summary.json"), "w"), indent=1)
    dig = os.path.join(src, "src_digest")
    summary["src_digest"] = open(dig).read().strip() if os.path.exists(dig) else None
    json.dump(summary, open(os.path.join(out_dir, f"{wl}_summary.json"), "w"), indent=1)
    json.dump({key: {"hbm_bytes_per_launch": summary["hbm_bytes_per_launch"], "valu_busy_frac": summary["valu_busy"],
                               "src_digest": summary["src_digest"],
                               "rocprof_avg_ns": summary["mean_launch_us"] * 1e3,
                               "profile": f"profiles/{tag}/{wl}_summary.json"}},
              open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w"), indent=1)
    print(wl, {k: summary[k] for k in ("launches_per_frame", "frame_kernel_us", "mean_launch_us",
                                       "hbm_bytes_per_launch", "valu_busy")})


if __name__ == "__main__":
    tag = sys.argv[1]
    for wl in sys.argv[2:] or ["c2_s1024", "c3_s1024_reflect", "c4_teapot", "c5_area_light"]:
        export(tag, wl)

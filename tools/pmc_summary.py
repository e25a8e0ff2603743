#!/usr/bin/env python3
"""Summarise a tools/gpu/prof.sh run (rocprofv3 kernel trace + PMC passes) for the
dominant kernel: per-launch averages of every counter, the kernel-trace duration,
and the HBM traffic figure bench.py reports (profiles/pmc_traffic.json).

usage: tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>/<tag>
"""
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "align_kernel<128, false>"


def per_launch(path):
    vals = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    out = {"kernel": KERNEL, "counters_per_launch": {}}
    for d in sorted(glob.glob(os.path.join(src, "pmc*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if os.path.exists(f):
            out["counters_per_launch"].update(per_launch(f))
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    for r in csv.DictReader(open(ks)):
        if KERNEL in r["Name"]:
            out["kernel_trace"] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                   "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))):
        if KERNEL in r["Kernel_Name"]:
            out["resources"] = {k: r[k] for k in ("LDS_Block_Size", "Scratch_Size", "VGPR_Count", "SGPR_Count",
                                                 "Grid_Size_X", "Workgroup_Size_X")}
            break
    c = out["counters_per_launch"]
    if "FETCH_SIZE" in c:
        # FETCH_SIZE / WRITE_SIZE are in KiB.  Uncorrected: the guide's x2 gfx950 correction is
        # calibrated for 16-B/lane streaming reads; these accesses are random 4-16 B gathers.
        fb = c["FETCH_SIZE"] * 1024
        wb = c.get("WRITE_SIZE", 0.0) * 1024
        out["hbm_bytes_per_launch"] = {"fetch": fb, "write": wb, "total": fb + wb}
        if "kernel_trace" in out:
            out["hbm_GBps"] = (fb + wb) / (out["kernel_trace"]["avg_ms"] / 1e3) / 1e9
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        out["wave_state"] = {k: round(c[k] / w, 4) for k in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                            "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                            "SQ_ACTIVE_INST_LDS") if k in c}
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    if "hbm_bytes_per_launch" in out:
        json.dump({"bytes_per_launch": out["hbm_bytes_per_launch"]["total"], "source": os.path.join(dst, "summary.json"),
                   "note": "rocprofv3 FETCH_SIZE+WRITE_SIZE (KiB x 1024) per align_kernel<128> launch, uncorrected",
                   "valu_insts_per_launch": out["counters_per_launch"].get("SQ_INSTS_VALU"),
                   "kernel_ms": out.get("kernel_trace", {}).get("avg_ms")},
                  open(os.path.join(os.path.dirname(dst.rstrip("/")), "..", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

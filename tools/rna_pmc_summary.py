#!/usr/bin/env python3
"""Summarise tools/gpu/rna_pmc.sh: per RNA kernel (align_kernel<256, false/true>, paired_kernel<256>)
the dispatches, their total rocprof duration, and every counter summed over the run's dispatches,
per call of snapgpu_rna_paired_align and per pair (the probe's calls x pairs); wave-state shares
(SQ_* / SQ_WAVE_CYCLES) and VALU lane utilisation.  HBM bytes are FETCH_SIZE / WRITE_SIZE (KiB)
x 1024, uncorrected.
usage: tools/rna_pmc_summary.py gpurun_out/rnapmc_<tag> profiles/<tag>/rna"""
import csv
import glob
import json
import os
import shutil
import sys

KERNELS = {"align256": "align_kernel<256, false>", "align256_ext": "align_kernel<256, true>",
           "paired256": "paired_kernel<256>"}


def kname(name):
    for k, v in KERNELS.items():
        if v in name:
            return k
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    probe = json.loads(open(os.path.join(src, "kt.json")).read().strip().splitlines()[-1])
    units = probe["calls"] * probe["pairs"]
    out = {"probe": probe, "kernels": {}}
    kt = glob.glob(os.path.join(src, "kt", "**", "run_kernel_trace.csv"), recursive=True)[0]
    tr = list(csv.DictReader(open(kt)))
    cols = tr[0].keys() if tr else []
    sc = next(c for c in cols if "Start" in c)
    ec = next(c for c in cols if "End" in c)
    for r in tr:
        k = kname(r["Kernel_Name"])
        if k:
            d = out["kernels"].setdefault(k, {"dispatches": 0, "ms": 0.0, "counters": {}})
            d["dispatches"] += 1
            d["ms"] += (int(r[ec]) - int(r[sc])) / 1e6
    for f in glob.glob(os.path.join(src, "pmc*", "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k and k in out["kernels"]:
                c = out["kernels"][k]["counters"]
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, d in out["kernels"].items():
        c = d["counters"]
        d["ms_per_call"] = d["ms"] / probe["calls"]
        d["per_pair"] = {x: v / units for x, v in c.items()}
        if "FETCH_SIZE" in c:
            d["per_pair"]["fetch_bytes"] = c["FETCH_SIZE"] * 1024 / units
        if "WRITE_SIZE" in c:
            d["per_pair"]["write_bytes"] = c["WRITE_SIZE"] * 1024 / units
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            d["wave_state"] = {x: round(c[x] / wc, 4) for x in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                 "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                                 "SQ_ACTIVE_INST_LDS") if x in c}
        if c.get("SQ_INSTS_VALU") and c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
            d["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    for f in glob.glob(os.path.join(src, "kt", "**", "run_kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
    print(json.dumps({k: {"ms_per_call": round(d["ms_per_call"], 2),
                          "per_pair": {x: round(v, 1) for x, v in d["per_pair"].items()}} for k, d in out["kernels"].items()}))


if __name__ == "__main__":
    main()

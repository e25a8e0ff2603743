#!/usr/bin/env python3
"""Summarise a tools/gpu/prof.sh run (rocprofv3 kernel trace + PMC passes).

Per kernel of interest: rocprof per-dispatch duration, the union of the dispatch intervals
(the bench's two HIP streams run launches concurrently), per-dispatch counter averages and
per-read figures (reads per dispatch from the bench line).  HBM bytes are FETCH_SIZE (KiB)
and WRITE_SIZE (KiB) x 1024, uncorrected; MI355X_MICROARCH.md calibrates FETCH_SIZE only for
16-B/lane streaming reads (x2), so copy_peak_kernel (known bytes, 16-B vector accesses) is
summarised beside them as the calibration point.  Writes profiles/<tag>/summary.json and,
keyed by the library's sha256, profiles/pmc_traffic.json (what bench.py reports as traffic).

usage: tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
"""
import csv
import glob
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"align": "align_kernel<128, false>", "lookup": "seed_lookup_kernel", "copy": "copy_peak_kernel",
           "paired": "paired_kernel<128>",
           "gather": "gather_peak_kernel", "cigar": "cigar_kernel", "align512": "align_kernel<512, false>"}


def kname(name):
    for k, v in KERNELS.items():
        if v in name:
            return k
    return None


def per_dispatch(path):
    vals = {}
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            d = vals.setdefault(k, {}).setdefault(r["Counter_Name"], {})
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def union(iv):
    iv.sort()
    tot, cs, ce = 0, None, None
    for b, e in iv:
        if ce is None or b > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = b, e
        elif e > ce:
            ce = e
    if ce is not None:
        tot += ce - cs
    return tot


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    bench = json.loads(open(os.path.join(src, "bench_kt.json")).readline())
    reads_per_launch = bench["roofline"]["reads_per_launch"]
    out = {"bench_line": os.path.join(dst, "bench_kt.json"), "lib_sha256": bench["roofline"]["lib_sha256"],
           "kernel_source_sha256": bench["roofline"].get("kernel_source_sha256"),
           "kernels": {}}
    shutil.copy(os.path.join(src, "bench_kt.json"), os.path.join(dst, "bench_kt.json"))
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(ks)):
        k = kname(r["Name"])
        if k:
            out["kernels"].setdefault(k, {})["rocprof_stats"] = {
                "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6, "min_ms": float(r["MinNs"]) / 1e6,
                "max_ms": float(r["MaxNs"]) / 1e6, "total_ms": float(r["TotalDurationNs"]) / 1e6}
    tr = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))))
    cols = tr[0].keys() if tr else []
    sc = next(c for c in cols if "Start" in c)
    ec = next(c for c in cols if "End" in c)
    iv = {}
    for r in tr:
        k = kname(r["Kernel_Name"])
        if k:
            iv.setdefault(k, []).append((int(r[sc]), int(r[ec])))
            if k == "align" and "resources" not in out:
                out["resources"] = {c: r[c] for c in ("LDS_Block_Size", "Scratch_Size", "VGPR_Count", "SGPR_Count",
                                                    "Grid_Size_X", "Workgroup_Size_X") if c in r}
    for k, v in iv.items():
        out["kernels"].setdefault(k, {})["trace"] = {"dispatches": len(v), "busy_union_ms": union(v) / 1e6,
                                                     "busy_ms_per_dispatch": union(v) / 1e6 / len(v)}
    cnt = {}
    for d in sorted(glob.glob(os.path.join(src, "pmc*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if os.path.exists(f):
            for k, cs in per_dispatch(f).items():
                cnt.setdefault(k, {}).update(cs)
    for k, c in cnt.items():
        e = out["kernels"].setdefault(k, {})
        e["counters_per_dispatch"] = c
        if "FETCH_SIZE" in c:
            e["hbm_bytes_per_dispatch_raw"] = {"fetch": c["FETCH_SIZE"] * 1024, "write": c.get("WRITE_SIZE", 0) * 1024}
        if "SQ_WAVE_CYCLES" in c:
            w = c["SQ_WAVE_CYCLES"]
            e["wave_state"] = {x: round(c[x] / w, 4) for x in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                                "SQ_ACTIVE_INST_LDS") if x in c}
        if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c and c["SQ_ACTIVE_INST_VALU"]:
            e["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    # seed_lookup_kernel on serialised streams (prof.sh serial_kt / serial_pmc): rocprof's average
    # dispatch duration is the kernel's own, FETCH_SIZE (KiB) per dispatch over it is its HBM rate
    sk = os.path.join(src, "serial_kt", "run_kernel_stats.csv")
    sp = os.path.join(src, "serial_pmc", "run_counter_collection.csv")
    if os.path.exists(sk) and os.path.exists(sp):
        dur = {kname(r["Name"]): float(r["AverageNs"]) / 1e9 for r in csv.DictReader(open(sk)) if kname(r["Name"])}
        fc = per_dispatch(sp)
        if "lookup" in dur and "lookup" in fc and "FETCH_SIZE" in fc["lookup"]:
            fb = fc["lookup"]["FETCH_SIZE"] * 1024
            shutil.copy(sk, os.path.join(dst, "kernel_stats_serial.csv"))
            out["kernels"]["lookup"]["serialised"] = {
                "avg_dispatch_ms": dur["lookup"] * 1e3, "fetch_bytes_per_dispatch_raw": fb,
                "fetch_GBps": fb / dur["lookup"] / 1e9, "frac_of_8TBps": fb / dur["lookup"] / 1e9 / 8000.0,
                "note": "SNAPGPU_OVERLAP=0: no align kernel shares the GPU with the lookup dispatches; FETCH_SIZE "
                        "uncorrected (MI355X_MICROARCH.md calibrates it for 16-B streaming reads only)"}
    a = out["kernels"].get("align", {})
    if "counters_per_dispatch" in a:
        c = a["counters_per_dispatch"]
        per_read = {x: c[x] / reads_per_launch for x in c}
        a["per_read"] = per_read
        hb = a.get("hbm_bytes_per_dispatch_raw", {})
        traffic = {"lib_sha256": out["lib_sha256"], "kernel_source_sha256": out["kernel_source_sha256"],
                   "kernel": KERNELS["align"], "reads_per_dispatch": reads_per_launch,
                   "hbm_bytes_per_read": (hb.get("fetch", 0) + hb.get("write", 0)) / reads_per_launch,
                   "fetch_bytes_per_read": hb.get("fetch", 0) / reads_per_launch,
                   "write_bytes_per_read": hb.get("write", 0) / reads_per_launch,
                   "valu_insts_per_read": per_read.get("SQ_INSTS_VALU"),
                   "salu_insts_per_read": per_read.get("SQ_INSTS_SALU"),
                   "branch_insts_per_read": per_read.get("SQ_INSTS_BRANCH"),
                   "lds_insts_per_read": per_read.get("SQ_INSTS_LDS"),
                   "vmem_insts_per_read": (per_read.get("SQ_INSTS_VMEM_RD") or 0) + (per_read.get("SQ_INSTS_VMEM_WR") or 0),
                   "smem_insts_per_read": per_read.get("SQ_INSTS_SMEM"),
                   # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md): x4 = shader cycles
                   "wave_cycles_per_read": 4 * per_read["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in per_read else None,
                   # share of the waves' lifetime (SQ_WAVE_CYCLES) each state takes: issuing VALU / any
                   # instruction, waiting on a counter (memory), waiting for a dependency to issue
                   "wave_state": a.get("wave_state"),
                   "source": os.path.join(dst, "summary.json"),
                   "note": "rocprofv3 FETCH_SIZE + WRITE_SIZE (KiB x 1024) per dispatch / reads per dispatch; "
                           "uncorrected (random 4-16 B gathers: the guide's x2 streaming factor does not apply)"}
        json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

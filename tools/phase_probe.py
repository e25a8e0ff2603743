#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of align_kernel on the bench workload.

Needs a library built with the timers compiled in (they cost SGPR spills, so the
production build leaves them out):
    MK='s/PHASE_TIMERS ?= 0/PHASE_TIMERS ?= 1/' tools/build_variant.sh phases ""   # -> libsnapgpu_phases.so
Run on the GPU box:
    SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_phases.so SNAPGPU_PHASES=1 python tools/phase_probe.py [--reads N]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
os.environ.setdefault("SNAPGPU_PHASES", "1")
import snapgpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, default=1_000_000)
ap.add_argument("--genome-bases", type=int, default=46_709_983)
ap.add_argument("--contigs", type=int, default=1)
ap.add_argument("--families", type=int, default=200)
args = ap.parse_args()
# C2 defaults; C3 (bench --workload c3): --genome-bases 3100000000 --contigs 25 --families 2000
g = snapgpu.Genome.synthetic(args.genome_bases, seed=2121, n_contigs=args.contigs, n_repeat_families=args.families)
reads = snapgpu.Reads.synthetic(g, args.reads, seed=99)
idx = snapgpu.GenomeIndex.build(g, 20, 16)
del g   # the index keeps its genome
al = snapgpu.BaseAligner(idx, device=0)
dev = al.upload(reads)
dev.run(); dev.synchronize()
al.phase_cycles(reset=True)
dev.run(); dev.synchronize()
ph = al.phase_cycles(reset=True)
ms = al.timing()["mainKernelMs"]
tot = sum(ph[k] for k in ("setup", "lookup", "insert", "score", "out"))
ph["cycles_per_read_total"] = tot
out = {"kernel_ms": ms, "reads": args.reads, "cycles_per_read": {k: ph[k] / args.reads for k in ph}}
out["share_of_wave_time"] = {k: round(ph[k] / tot, 4) for k in ("setup", "lookup", "insert", "score", "pop",
                                                                 "stage", "lv_fwd", "lv_rev", "apply", "writeback", "out",
                                                                 "select", "fetch", "passloop", "rank", "candlist", "succ",
                                                                 "nearby", "prob", "fails", "succ_tail")}
n = max(ph["n_succ"], 1)
out["cycles_per_success"] = {k: round(ph[k] / n, 1) for k in ("succ", "nearby", "prob", "succ_tail")}
out["cycles_per_pass"] = {k: round(ph[k] / max(ph["n_pass"], 1), 1) for k in ("passloop", "stage", "lv_fwd", "lv_rev", "apply", "fails", "succ")}
out["forced"] = {"passes_per_read": ph["n_pass_forced"] / args.reads, "passloop_cycles_per_read": ph["passloop_forced"] / args.reads,
                 "candidates_per_read": ph["n_cand_forced"] / args.reads,
                 "filter_results_per_read": ph["n_filter_results"] / args.reads,
                 "lv_candidates_per_read": ph["n_lv_forced"] / args.reads,
                 "lv_candidates_with_filter_distances_per_read": ph["n_lv_forced_known"] / args.reads,
                 "lv_unknown_at_k_le_5_per_read": ph["n_lv_forced_unknown_lowk"] / args.reads,
                 "lv_unknown_not_first_of_element_per_read": ph["n_lv_forced_unknown_second"] / args.reads,
                 "nonforced_passes_per_read": (ph["n_pass"] - ph["n_pass_forced"]) / args.reads,
                 "nonforced_passloop_cycles_per_read": (ph["passloop"] - ph["passloop_forced"]) / args.reads}
out["heavy_reads"] = {"def": ">= 64 candidate elements", "share_of_reads": ph["n_heavy_reads"] / args.reads,
                      "share_of_cycles": ph["heavy_read_cycles"] / max(1, ph["read_cycles"])}
out["pass_overhead_per_pass"] = round((ph["passloop"] - ph["stage"] - ph["lv_fwd"] - ph["lv_rev"] - ph["apply"]) / max(ph["n_pass"], 1), 1)
print(json.dumps(out, indent=1))

#!/usr/bin/env python3
"""Diagnostic: the paired-end aligner on the C2 genome (wgsim-like 2 x 101 pairs), timing of the
intersect-only and chimeric calls; run under rocprofv3 --kernel-trace --stats for kernel times."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
import snapgpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=500_000)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1, n_repeat_families=200)
idx = snapgpu.GenomeIndex.build(g, 20, 16)
r0, r1 = snapgpu.Reads.synthetic_pairs(idx.genome_handle(), args.pairs, seed=7, read_length=101)
pa = snapgpu.PairedAligner(idx)
pa.align(r0, r1)
for what, fn in (("intersect", pa.intersect), ("chimeric", pa.align)):
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        fn(r0, r1)
        ts.append(time.perf_counter() - t0)
    print(what, "ms", [round(t * 1000, 2) for t in ts], "reads/s", round(2 * args.pairs / min(ts) / 1e6, 2), "M",
          flush=True)

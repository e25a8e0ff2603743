#!/usr/bin/env python3
"""CPU-baseline calibration: the C restatement (oracle/snap_oracle.c,
bench.py's cpu_baseline) against the reference's own BaseAligner (oracle/_ref/ref_harness,
built from /root/reference by oracle/Makefile.ref) on the same genome, index and reads,
one thread each.  Container only (needs oracle/_ref).  Prints reads/s for both and the
ratio restatement / reference: >= 1 means the bench's GPU/CPU speed-up is not inflated.

    python3 tools/calibrate_cpu.py [--genome-bases N] [--reads N]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "snap-rnaseq_amd"), os.path.join(ROOT, "tests")]
import snapgpu  # noqa: E402
from oracle_ffi import oracle_align  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--genome-bases", type=int, default=46_709_983)
ap.add_argument("--reads", type=int, default=20_000)
args = ap.parse_args()
work = tempfile.mkdtemp(prefix="calib_")
g = snapgpu.Genome.synthetic(args.genome_bases, seed=2121, n_contigs=1, n_repeat_families=200)
fa = os.path.join(work, "g.fa")
g.write_fasta(fa)
reads = snapgpu.Reads.synthetic(g, args.reads, seed=99)
fq = os.path.join(work, "r.fq")
reads.write_fastq(fq)
idxdir = os.path.join(work, "idx")
subprocess.run([os.path.join(ROOT, "oracle", "_ref", "snap-rna"), "index", fa, idxdir], check=True,
               capture_output=True)
empty = os.path.join(work, "empty.fq")
open(empty, "w").close()
t0 = time.perf_counter()   # index load alone, subtracted below
subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness"), "align", idxdir, empty], check=True,
               capture_output=True)
t_load = time.perf_counter() - t0
t0 = time.perf_counter()
subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness"), "align", idxdir, fq], check=True,
               capture_output=True)
t_ref = time.perf_counter() - t0 - t_load
idx = snapgpu.GenomeIndex.load(idxdir)   # the reference's own index files
p = snapgpu.default_params()
t0 = time.perf_counter()
oracle_align(idx, reads, p, n_threads=1)
t_orc = time.perf_counter() - t0
print(f"reference BaseAligner (1 thread, index load {t_load:.2f} s excluded): {args.reads / t_ref:,.0f} reads/s")
print(f"C restatement (1 thread): {args.reads / t_orc:,.0f} reads/s")
print(f"ratio restatement / reference: {t_ref / t_orc:.2f}")

"""Batch-size scaling of the RNA aligners (bench extras.rna_paired workload shape, C2 genome):
kernel and call time of the transcriptome aligner (plain AlignRead, 2 x 150 b pairs' end 0)
and of the chimeric paired aligner over 25k..400k pairs.  A fit time = fixed + n * marginal
separates the per-call cost (launches, copies, the persistent kernels' tail) from the per-read
cost.
  python tools/rna_tail_probe.py"""
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import snapgpu  # noqa: E402
from rna_synth import synth_rna_workload  # noqa: E402


def best(fn, k=3):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


def main():
    g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    pa = snapgpu.PairedAligner(idx, device=0)
    ta = None
    rows = []
    for n in (25_000, 50_000, 100_000, 200_000, 400_000):
        work = tempfile.mkdtemp(prefix="rna_tail_")
        try:
            gtf_path, fq0, fq1, _ = synth_rna_workload(idx.genome_handle(), work, n_pairs=n)
            if ta is None:   # one transcriptome (the GTF does not depend on n)
                gtf = snapgpu.Gtf.load(gtf_path)
                tfa = os.path.join(work, "transcriptome.fa")
                gtf.write_transcriptome(idx.genome_handle(), tfa)
                tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 16)
                ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8,
                                         extraSearchDepth=2)
            r0, r1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)
            r0.clip(3)
            r1.clip(3)
            row = {"pairs": n}
            row["t_call_ms"] = best(lambda: ta.AlignReads(r0))
            t = ta.timing()
            row["t_kernel_ms"] = t["spillKernelMs"] + t["mainKernelMs"]
            row["t_lookup_ms"] = t["lookupKernelMs"]
            row["paired_call_ms"] = best(lambda: pa.align(r0, r1))
            row["intersect_ms"] = best(lambda: pa.intersect(r0, r1))
            rows.append(row)
            print(row, flush=True)
        finally:
            shutil.rmtree(work, ignore_errors=True)
    n = np.array([r["pairs"] for r in rows], dtype=float)
    fit = {}
    for k in ("t_call_ms", "t_kernel_ms", "paired_call_ms", "intersect_ms"):
        y = np.array([r[k] for r in rows])
        m, c = np.polyfit(n, y, 1)
        fit[k] = {"fixed_ms": round(float(c), 2), "ms_per_100k": round(float(m) * 1e5, 2)}
    print({"fit": fit}, flush=True)


if __name__ == "__main__":
    main()

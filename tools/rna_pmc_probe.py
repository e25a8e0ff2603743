"""The bench's RNA paired leg (extras.rna_paired workload: C2 genome, 2,000-gene GTF, 2 x 150 bp
pairs) run CALLS times through snapgpu.rna_paired_align, for rocprofv3 kernel-trace / PMC passes
(tools/gpu/rna_pmc.sh).  Index and workload preparation happen before the first call; every
kernel dispatch of align_kernel<256,*> / paired_kernel<256> in the run belongs to the CALLS calls.
  python tools/rna_pmc_probe.py [pairs] [calls]"""
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import snapgpu  # noqa: E402
from rna_synth import synth_rna_workload  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    work = tempfile.mkdtemp(prefix="snapgpu_rnapmc_")
    try:
        gtf_path, fq0, fq1, info = synth_rna_workload(idx.genome_handle(), work, n_pairs=n)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 16)
        pa = snapgpu.PairedAligner(idx, device=0)
        ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2, device=0)
        r0, r1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)
        ts = []
        for _ in range(calls):
            gtf.reset_counts()
            c0 = time.perf_counter()
            snapgpu.rna_paired_align(pa, ta, gtf, r0, r1)
            ts.append(time.perf_counter() - c0)
        print(json.dumps({"pairs": n, "calls": calls, "call_ms": [round(t * 1e3, 1) for t in ts]}))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

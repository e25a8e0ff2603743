"""align_kernel<256> on 2 x 150 RNA work vs align_kernel<128>: per-call kernel time and per-read work
(elements, LV-scored locations, hit words) for
  (a) C2 wgsim reads of 100 b and 150 b at the default single-end parameters,
  (b) the same at the RNA transcriptome / paired parameters (maxHits 16000, maxK 15, 8 seeds),
  (c) bench extras.rna_paired's transcriptome reads (end 0) on the transcriptome index.
  python tools/probe256.py [n_reads]"""
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import snapgpu  # noqa: E402
from rna_synth import synth_rna_workload  # noqa: E402


def stats(al, reads, tag):
    res = al.AlignReads(reads)
    ks, sp = [], []
    for _ in range(3):
        al.AlignReads(reads, out=res)
        t = al.timing()
        ks.append(t["mainKernelMs"])
        sp.append(t["spillKernelMs"])
    q = lambda a: [int(np.percentile(a, p)) for p in (50, 90, 99, 99.9)] + [int(a.max())]
    print(f"{tag:38s} n={len(res)} pass1_ms={min(ks):.2f} pass2+3_ms={min(sp):.2f} "
          f"elems p50/90/99/99.9/max={q(res['nElements'])} scored={q(res['nLocationsScored'])} "
          f"hitwords={q(res['nHitWords'])} mean_scored={res['nLocationsScored'].mean():.1f} "
          f"mean_elems={res['nElements'].mean():.1f}", flush=True)
    return res


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    rna = dict(maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    d = snapgpu.BaseAligner(idx, device=0)
    r = snapgpu.BaseAligner(idx, device=0, **rna)
    for L in (100, 150):
        reads = snapgpu.Reads.synthetic(idx.genome_handle(), n, seed=99, read_length=L)
        stats(d, reads, f"C2 {L} b, defaults")
        stats(r, reads, f"C2 {L} b, RNA params")
    work = tempfile.mkdtemp(prefix="probe256_")
    try:
        gtf_path, fq0, fq1, info = synth_rna_workload(idx.genome_handle(), work, n_pairs=n)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 16)
        ta = snapgpu.BaseAligner(tidx, device=0, **rna)
        r0 = snapgpu.Reads.from_fastq(fq0)
        res = stats(ta, r0, "RNA transcriptome end 0")
        stats(r, r0, "RNA genome end 0 (RNA params)")
        heavy = np.argsort(res["nLocationsScored"])[::-1][:5]
        print("heaviest transcriptome reads:", [(int(i), int(res["nElements"][i]), int(res["nLocationsScored"][i]),
                                               int(res["nHitWords"][i])) for i in heavy], flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

"""Sub-batch pipeline of the RNA paired path (snapgpu_rna_paired_align, SNAPGPU_RNA_SUBBATCH): the
bench extras.rna_paired workload (100k 2 x 150 pairs, C2 genome, 2,000-gene GTF) in 1, 2, 3 and 4
sub-batches, best of 3 calls each, with the stage times of the best call.
  python tools/rna_sub_probe.py [n_pairs] [sub-batch counts, e.g. 1,2]"""
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
    g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    work = tempfile.mkdtemp(prefix="rna_sub_")
    try:
        gtf_path, fq0, fq1, _ = synth_rna_workload(idx.genome_handle(), work, n_pairs=n)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 16)
        pa = snapgpu.PairedAligner(idx, device=0)
        ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
        R0, R1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)
        gtf.reset_counts()
        snapgpu.rna_paired_align(pa, ta, gtf, R0, R1)   # warm-up
        counts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 3, 4]
        for subs in counts:
            os.environ["SNAPGPU_RNA_SUBBATCH"] = str((n + subs - 1) // subs)
            best = None
            for _ in range(3):
                gtf.reset_counts()
                t0 = time.perf_counter()
                _, st = snapgpu.rna_paired_align(pa, ta, gtf, R0, R1)
                dt = (time.perf_counter() - t0) * 1e3
                if best is None or dt < best[0]:
                    best = (dt, st)
            os.environ.pop("SNAPGPU_RNA_SUBBATCH", None)
            st = best[1]
            print({"sub_batches": subs, "ms": round(best[0], 1), "M_reads_per_s": round(2 * n / best[0] / 1e3, 3),
                   "stage_ms": {k: round(st[k], 1) for k in ("prepMs", "alignMs", "filterMs", "seedMs", "countMs",
                                                            "cigarMs", "cigarGpuMs", "spliceMs", "writeMs", "wallMs")}},
                  flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

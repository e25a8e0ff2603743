"""Stage timing of the RNA paired path (bench extras.rna_paired workload) on one GPU:
transcriptome AlignReadsEx per end (1000 multi-hits), the chimeric paired aligner, the
intersecting kernel alone, the whole snapgpu_rna_paired_align call, and snapgpu_single_align over end 0.
  python tools/rna_probe.py [n_pairs]"""
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


def best(fn, k=3):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 1)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    work = tempfile.mkdtemp(prefix="rna_probe_")
    try:
        gtf_path, fq0, fq1, info = synth_rna_workload(idx.genome_handle(), work, n_pairs=n)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 16)
        pa = snapgpu.PairedAligner(idx, device=0)
        ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
        r0, r1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)
        r0.clip(3)
        r1.clip(3)
        out = {"pairs": n}
        out["transcriptome_ex_end0_ms"] = best(lambda: ta.AlignReadsEx(r0, maxHitsToGet=1000))
        out["transcriptome_ex_timing"] = {k: round(v, 2) if isinstance(v, float) else v for k, v in ta.timing().items()
                                          if k in ("mainKernelMs", "spillKernelMs", "lookupKernelMs", "nSpilled", "nByteReads", "nArenaOverflow")}
        out["transcriptome_ex0_end0_ms"] = best(lambda: ta.AlignReadsEx(r0, maxHitsToGet=0))
        out["transcriptome_plain_end0_ms"] = best(lambda: ta.AlignReads(r0))
        out["transcriptome_plain_timing"] = {k: round(v, 2) if isinstance(v, float) else v for k, v in ta.timing().items()
                                             if k in ("mainKernelMs", "spillKernelMs", "lookupKernelMs", "nSpilled", "nByteReads", "nArenaOverflow")}
        out["paired_align_ms"] = best(lambda: pa.align(r0, r1))
        out["paired_intersect_ms"] = best(lambda: pa.intersect(r0, r1))
        ga = snapgpu.BaseAligner(idx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
        out["genome_single_end0_ms"] = best(lambda: ga.AlignReads(r0))
        R0, R1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)

        def full():
            gtf.reset_counts()
            _, st = snapgpu.rna_paired_align(pa, ta, gtf, R0, R1)
            out["stage_ms"] = {k: round(st[k], 1) for k in ("prepMs", "alignMs", "filterMs", "seedMs", "countMs", "cigarMs",
                                                                    "cigarGpuMs", "spliceMs", "writeMs", "wallMs")}
        os.environ["SNAPGPU_RNA_SUBBATCH"] = str(n)   # one batch (the default splits >= 40k pairs in two)
        out["rna_paired_align_ms"] = best(full)
        # the same call pipelined over two sub-batches (stage A of the second overlaps stage B of the first)
        os.environ["SNAPGPU_RNA_SUBBATCH"] = str((n + 1) // 2)
        out["rna_paired_align_2sub_ms"] = best(full)
        out["stage_ms_2sub"] = out.pop("stage_ms")
        del os.environ["SNAPGPU_RNA_SUBBATCH"]
        full()
        # the single-end product path (snap-rna single) over end 0
        S0 = snapgpu.Reads.from_fastq(fq0)
        sam = os.path.join(work, "single.sam")

        def single():
            gtf.reset_counts()
            st = snapgpu.single_align(ga, ta, gtf, S0, sam)
            out["single_stage_ms"] = {k: round(v, 1) for k, v in st.items() if k.endswith("Ms")}
        out["single_align_ms"] = best(single)
        print(out, flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

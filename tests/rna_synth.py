"""Synthetic RNA-seq workload (BASELINE configs[4] shape, no GRCh38 / GENCODE offline): a GTF
of multi-exon genes with alternative transcripts laid on a genome, and 2 x L read pairs drawn
from the transcripts' spliced mRNAs (junction-crossing fragments), from pre-mRNA spans (what the
reference's transcriptome index holds, GTFReader::BuildTranscriptome), from intergenic sequence,
chimeras of two genes, and noise.  Deterministic (numpy PCG64 with fixed seeds).  Used by
bench.py's `extras.rna_paired` leg and the GPU tests of the RNA paired path."""
import ctypes as C
import os

import numpy as np

COMP = bytes.maketrans(b"ACGTNn", b"TGCANN")


def _rc(b):
    return b.translate(COMP)[::-1]


def synth_rna_workload(genome_handle, workdir, n_genes=2000, n_pairs=100_000, read_len=150, seed=5,
                       sub_rate=0.005):
    """-> (gtf_path, fastq0, fastq1, info).  genome_handle: a snapgpu genome handle
    (GenomeIndex.genome_handle())."""
    import snapgpu
    from snapgpu import lib
    L = lib()
    rng = np.random.default_rng(seed)
    base = L.snapgpu_genome_bases(genome_handle)
    nb = L.snapgpu_genome_nbases(genome_handle)
    npc = L.snapgpu_genome_npieces(genome_handle)
    offs = [L.snapgpu_genome_piece_offset(genome_handle, i) for i in range(npc)] + [nb]
    names = [L.snapgpu_genome_piece_name(genome_handle, i).decode() for i in range(npc)]
    seqs = [C.string_at(base + offs[i], offs[i + 1] - offs[i]).upper() for i in range(npc)]
    # genes: 2-8 exons of 80-400 bp, introns of 200-4000 bp, 1-3 transcripts (exon subsets)
    lines, spliced, premrna = [], [], []
    for g in range(n_genes):
        c = int(rng.integers(npc))
        span_max = len(seqs[c]) - 2000
        nex = int(rng.integers(2, 9))
        ex_len = rng.integers(80, 401, nex)
        in_len = rng.integers(200, 4001, nex - 1)
        total = int(ex_len.sum() + in_len.sum())
        if total >= span_max:
            continue
        p = int(rng.integers(1000, span_max - total))
        exons = []
        for e in range(nex):
            exons.append((p, p + int(ex_len[e]) - 1))
            p += int(ex_len[e]) + (int(in_len[e]) if e < nex - 1 else 0)
        strand = "+-"[g % 2]
        lines.append(f"{names[c]}\tsynth\tgene\t{exons[0][0]}\t{exons[-1][1]}\t.\t{strand}\t.\t"
                     f'gene_id "G{g}"; gene_name "GENE{g}";')
        for t in range(int(rng.integers(1, 4))):
            use = exons if t == 0 else [x for k, x in enumerate(exons)
                                        if k == 0 or k == nex - 1 or rng.random() < 0.6]
            for a, b in use:
                lines.append(f"{names[c]}\tsynth\texon\t{a}\t{b}\t.\t{strand}\t.\tgene_id \"G{g}\"; "
                             f"transcript_id \"T{g}.{t}\"; gene_name \"GENE{g}\"; transcript_name \"GENE{g}-{t}\";")
            spliced.append(b"".join(seqs[c][a - 1:b] for a, b in use))
            premrna.append(seqs[c][use[0][0] - 1:use[-1][1]])
    gtf_path = os.path.join(workdir, "synth.gtf")
    with open(gtf_path, "w") as f:
        f.write("\n".join(lines) + "\n")
    # pairs
    kinds = rng.random(n_pairs)
    frag = rng.integers(read_len + 50, read_len + 350, n_pairs)
    out0, out1 = [], []
    kind_counts = {}
    for i in range(n_pairs):
        u = kinds[i]
        F = int(frag[i])
        if u < 0.65:
            src, k = spliced[int(rng.integers(len(spliced)))], "spliced"
        elif u < 0.78:
            src, k = premrna[int(rng.integers(len(premrna)))], "premrna"
        elif u < 0.90:
            c = int(rng.integers(npc))
            p = int(rng.integers(0, len(seqs[c]) - F - 1))
            src, k = seqs[c][p:p + F], "genomic"
        elif u < 0.95:
            a = spliced[int(rng.integers(len(spliced)))]
            b = spliced[int(rng.integers(len(spliced)))]
            src, k = a[:F // 2] + b[-(F - F // 2):], "chimeric"
        else:
            src, k = bytes(rng.choice(list(b"ACGT"), F).astype(np.uint8)), "random"
        kind_counts[k] = kind_counts.get(k, 0) + 1
        if len(src) < read_len:
            src = src + bytes(rng.choice(list(b"ACGT"), read_len - len(src)).astype(np.uint8))
        F = min(F, len(src))
        p = int(rng.integers(0, len(src) - F + 1))
        f = src[p:p + F]
        if rng.random() < 0.5:
            f = _rc(f)
        out0.append(f[:read_len])
        out1.append(_rc(f[len(f) - read_len:]))
    # substitutions, in bulk
    for reads in (out0, out1):
        buf = np.frombuffer(b"".join(reads), dtype=np.uint8).copy()
        m = rng.random(len(buf)) < sub_rate
        buf[m] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, int(m.sum()))]
        buf[buf == ord("n")] = ord("N")
        data = buf.tobytes()
        pos = 0
        for j in range(len(reads)):
            n = len(reads[j])
            reads[j] = data[pos:pos + n]
            pos += n
    paths = []
    for mate, reads in ((1, out0), (2, out1)):
        path = os.path.join(workdir, f"rna_{mate}.fq")
        with open(path, "wb") as f:
            for i, r in enumerate(reads):
                f.write(b"@rp%d/%d\n%s\n+\n%s\n" % (i, mate, r, b"I" * len(r)))
        paths.append(path)
    info = {"genes": n_genes, "transcripts": len(spliced), "pairs": n_pairs, "read_len": read_len,
            "kinds": kind_counts}
    return gtf_path, paths[0], paths[1], info


def synth_single_reads(genome_handle, workdir, n_reads=1_000_000, read_len=100):
    """The single-end workload of bench.py's `extras.single_e2e` (`snap-rna single`) and of
    tests/golden/make_golden.py --only-single-bench: synth_rna_workload's fragments at 100 bp, whose
    first ends are the reads; the GTF is the RNA paired leg's (the genes are drawn before the reads).
    -> (gtf_path, fastq, info)."""
    gtf, fq0, fq1, info = synth_rna_workload(genome_handle, workdir, n_pairs=n_reads, read_len=read_len)
    os.unlink(fq1)
    info = dict(info, reads=info.pop("pairs"))
    return gtf, fq0, info

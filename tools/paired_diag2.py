"""Does the intersecting aligner's `tight` run go wrong after another paired aligner ran in the
same process?  Sequences: (a) tight alone; (b) default intersect, free, tight; (c) default aligner
created and freed without a call, tight; (d) default intersect kept alive, tight; each tight call
compared with the reference fixture (and the first bad pairs printed)."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import snapgpu  # noqa: E402
from golden_common import PAIRED_RUNS  # noqa: E402
from oracle_ffi import paired_tsv_rows, ref_paired_rows  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
r0 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_1.fq"))
r1 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_2.fq"))
want = {run: ref_paired_rows(os.path.join(G, f"expected_paired_{run}.tsv"))[0] for run in PAIRED_RUNS}


def mk(run):
    d = PAIRED_RUNS[run]
    return snapgpu.PairedAligner(idx, maxHits=d["maxHits"], maxK=d["maxK"], maxSeedsToUse=d["numSeeds"],
                                 extraSearchDepth=d["extra"], minSpacing=d["minSpacing"], maxSpacing=d["maxSpacing"],
                                 maxBigHits=d["maxBigHits"])


def check(tag, run, pa):
    got = pa.intersect(r0, r1)
    rows = paired_tsv_rows(got, chimeric=False)
    bad = [i for i, (g, w) in enumerate(zip(rows, want[run])) if g != w]
    print(f"{tag:28s} {run}: {len(bad)} differ" + (f", first {bad[:6]}" if bad else ""), flush=True)
    for i in bad[:2]:
        print(f"    got  {rows[i]} flags {int(got['flags'][i]):#x} scored {int(got['nLocationsScored'][i])}\n"
              f"    want {want[run][i]}", flush=True)
    return len(bad)


total = 0
total += check("a: tight alone", "tight", mk("tight"))
for rep in range(2):
    pa = mk("default"); check("b: default", "default", pa); del pa; gc.collect()
    total += check("b: tight after default", "tight", mk("tight"))
    pa = mk("default"); del pa; gc.collect()
    total += check("c: tight after created default", "tight", mk("tight"))
    keep = mk("default"); check("d: default (kept)", "default", keep)
    total += check("d: tight beside default", "tight", mk("tight"))
    del keep; gc.collect()
    pa = mk("wide"); check("e: wide", "wide", pa); del pa; gc.collect()
    total += check("e: tight after wide", "tight", mk("tight"))
print("TOTAL_BAD_TIGHT", total)

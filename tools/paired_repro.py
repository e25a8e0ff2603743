"""Repeat the intersecting paired aligner of tests/test_paired.py (run `tight`, 2,400 pairs over
small.fa) in one process and compare every call with the reference fixture: K fresh aligners (each
builds its own bucket image) x M calls each.  Prints the pairs that differ per call, and for the
first differing call the lookups of its pairs' seeds through both device lookups."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import snapgpu  # noqa: E402
from golden_common import PAIRED_RUNS  # noqa: E402
from oracle_ffi import paired_tsv_rows, ref_paired_rows  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
M = int(sys.argv[2]) if len(sys.argv) > 2 else 3
run = sys.argv[3] if len(sys.argv) > 3 else "tight"
idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
r0 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_1.fq"))
r1 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_2.fq"))
want, _ = ref_paired_rows(os.path.join(G, f"expected_paired_{run}.tsv"))
d = PAIRED_RUNS[run]
bad_total = 0
for k in range(K):
    pa = snapgpu.PairedAligner(idx, maxHits=d["maxHits"], maxK=d["maxK"], maxSeedsToUse=d["numSeeds"],
                               extraSearchDepth=d["extra"], minSpacing=d["minSpacing"], maxSpacing=d["maxSpacing"],
                               maxBigHits=d["maxBigHits"])
    for m in range(M):
        got = pa.intersect(r0, r1)
        rows = paired_tsv_rows(got, chimeric=False)
        bad = [i for i, (g, w) in enumerate(zip(rows, want)) if g != w]
        bad_total += len(bad)
        print(f"aligner {k} call {m}: {len(bad)} pairs differ" + (f", first {bad[:8]}" if bad else ""), flush=True)
        if bad:
            for i in bad[:3]:
                print("   got ", rows[i], "\n   want", want[i], flush=True)
    del pa
print("TOTAL_BAD", bad_total)

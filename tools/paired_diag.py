"""Diagnose the intersecting aligner's `tight` disagreement: the reference fixture against the full
grid and against one wave (SNAPGPU_PAIRED_GRID=1), twice each, with the first differing pairs' fields."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import snapgpu  # noqa: E402
from golden_common import PAIRED_RUNS  # noqa: E402
from oracle_ffi import paired_tsv_rows, ref_paired_rows  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
run = sys.argv[1] if len(sys.argv) > 1 else "tight"
idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
r0 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_1.fq"))
r1 = snapgpu.Reads.from_fastq(os.path.join(G, "paired_2.fq"))
want, _ = ref_paired_rows(os.path.join(G, f"expected_paired_{run}.tsv"))
d = PAIRED_RUNS[run]


def once(grid):
    if grid:
        os.environ["SNAPGPU_PAIRED_GRID"] = str(grid)
    else:
        os.environ.pop("SNAPGPU_PAIRED_GRID", None)
    pa = snapgpu.PairedAligner(idx, maxHits=d["maxHits"], maxK=d["maxK"], maxSeedsToUse=d["numSeeds"],
                               extraSearchDepth=d["extra"], minSpacing=d["minSpacing"], maxSpacing=d["maxSpacing"],
                               maxBigHits=d["maxBigHits"])
    got = pa.intersect(r0, r1)
    rows = paired_tsv_rows(got, chimeric=False)
    bad = [i for i, (g, w) in enumerate(zip(rows, want)) if g != w]
    return rows, bad, got


res = {}
for name, grid in (("full_a", 0), ("one_a", 1), ("full_b", 0), ("one_b", 1), ("two", 2), ("seven", 7)):
    rows, bad, got = once(grid)
    res[name] = (rows, bad, got)
    print(f"{name:7s} grid={grid}: {len(bad)} pairs differ from the reference" + (f", first {bad[:10]}" if bad else ""), flush=True)
for name, (rows, bad, got) in res.items():
    for i in bad[:3]:
        print(f"  {name} pair {i}: got  {rows[i]}\n  {' ' * len(name)}          want {want[i]}\n  flags {got['flags'][i]:#x}", flush=True)
    if bad:
        break

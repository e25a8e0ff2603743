"""Shared definitions for the golden fixtures (tests/golden/) and their tests."""
import hashlib

# Parameter sets: (maxHits, maxK, numSeeds, extraSearchDepth) as the reference
# harness takes them (oracle/ref_harness.cpp mode_align).
PARAM_SETS = {
    "default": dict(maxHits=300, maxK=14, numSeeds=25, extra=2),
    "h16": dict(maxHits=16, maxK=14, numSeeds=25, extra=2),
    "k5": dict(maxHits=300, maxK=5, numSeeds=25, extra=1),
    "s4": dict(maxHits=50, maxK=8, numSeeds=4, extra=0),
    "k20": dict(maxHits=300, maxK=20, numSeeds=40, extra=5),
}

# C1: the reference's CPU-runnable config (BASELINE.json configs[0]): 1 Mb, 10k reads.
C1 = dict(name="C1",
          genome=dict(total_bases=1_000_000, seed=2121, n_contigs=1, n_repeat_families=60),
          reads=dict(n_reads=10_000, seed=99))
# C2: chr21-sized (46,709,983 bp) repeat-rich genome, 1M reads (configs[1], the bench workload).
C2 = dict(name="C2",
          genome=dict(total_bases=46_709_983, seed=2121, n_contigs=1, n_repeat_families=200),
          reads=dict(n_reads=1_000_000, seed=99))


def params_to_aligner_kwargs(p):
    return dict(maxHitsToConsider=p["maxHits"], maxK=p["maxK"], maxSeedsToUse=p["numSeeds"],
                extraSearchDepth=p["extra"])


def ref_tsv_to_canonical(text):
    """ref_harness align output (doubles as C %a) -> canonical lines (doubles as IEEE bits)."""
    import struct
    out = []
    for line in text.splitlines():
        x = line.split("\t")
        bits = [struct.unpack("<Q", struct.pack("<d", float.fromhex(v)))[0] for v in x[9:11]]
        out.append("\t".join(x[:9]) + f"\t{bits[0]:016x}\t{bits[1]:016x}")
    return "\n".join(out) + "\n"


def ref_tsvx_to_canonical(text):
    """ref_harness alignx output -> canonical lines (align columns as above + nFound + hits)."""
    out = []
    for line in text.splitlines():
        x = line.split("\t")
        out.append(ref_tsv_to_canonical("\t".join(x[:11])).rstrip("\n") + "\t" + "\t".join(x[11:13]))
    return "\n".join(out) + "\n"


# multi-hit / windowed-search fixture runs: name -> (maxHitsToGet, PARAM_SETS key)
MULTIHIT_RUNS = {"mh8": (8, "default"), "mh1": (1, "k5"), "mh64": (64, "h16")}

# ref_harness paired runs (PairedAligner.cpp:462-482).  "default" = the paired CLI defaults
# (AlignerOptions.cpp:73-77, PairedAligner.cpp:57-58,231-235): maxHits 16000, maxDist 15,
# 8 seeds, extraSearchDepth 2, spacing 50..1000, intersecting maxBigHits 16000.
PAIRED_RUNS = {
    "default": dict(maxHits=16000, maxK=15, numSeeds=8, extra=2, minSpacing=50, maxSpacing=1000, maxBigHits=16000),
    "tight": dict(maxHits=300, maxK=8, numSeeds=4, extra=1, minSpacing=100, maxSpacing=500, maxBigHits=300),
    "wide": dict(maxHits=2000, maxK=20, numSeeds=12, extra=3, minSpacing=0, maxSpacing=3000, maxBigHits=64),
}


def digest(text):
    return hashlib.sha256(text.encode()).hexdigest()

"""The device bucket image of the seed tables (csrc/bucket_table.h).

The aligner re-lays SNAPHashTable's key -> (value1, value2) map (HashTable.h:74-105) into 64-B
buckets when it is created; every device lookup goes through that image.  Exactness rests on the
map being the reference's, so these tests check device lookups, by both lookup forms (lane per
seed: seed_lookup_kernel / paired kernel; whole wave per seed: align_kernel / CharacterizeSeeds):

* against the reference's own lookupSeed fixture (tests/golden/expected_lookups.tsv, written by the
  compiled reference, GenomeIndex.cpp:971-1086), on our index and on the index the reference built;
* against the host lookupSeed (index.cpp, itself pinned to that fixture) on present, absent and
  popular seeds of a 1 Mb repeat-rich genome and at seed lengths 16 and 25 (1 and 262,144 tables);
* the image's own figures: every key the reference table can return is held, lines per lookup.
"""
import os
import tarfile

import numpy as np
import pytest

import snapgpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
M64 = (1 << 64) - 1


def _fixture_rows(out):
    rows = []
    for o in out:
        nf, nr, hf, hr, ff, fr = (int(x) for x in o)
        rows.append(f"{nf}\t{nr}\t{hf}\t{hr}\t{ff if nf else -1}\t{fr if nr else -1}")
    return rows


def _host_rows(index, seeds, cap=1 << 16):
    rows = []
    for s in seeds:
        f, r, (nf, nr) = index.lookupSeed(s, cap=cap)
        assert nf <= cap and nr <= cap
        sums = []
        for hits in (f, r):
            acc = 0
            for h in hits:
                acc = (acc * 1000003 + h) & M64
            sums.append(acc)
        rows.append(f"{nf}\t{nr}\t{sums[0]}\t{sums[1]}\t{f[0] if nf else -1}\t{r[0] if nr else -1}")
    return rows


def _seed_set(g, seed_len, n_present, n_random, seed=5):
    """g: genome bytes"""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n_present:   # seeds at random genome positions (ACGT only), either strand
        p = int(rng.integers(0, len(g) - seed_len))
        s = g[p:p + seed_len].upper()
        if set(s) <= set(b"ACGT"):
            if rng.integers(0, 2):
                s = s[::-1].translate(bytes.maketrans(b"ACGT", b"TGCA"))
            out.append(s.decode())
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    for _ in range(n_random):   # random seeds: almost all absent
        out.append(acgt[rng.integers(0, 4, seed_len)].tobytes().decode())
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gpu_lookups_match_reference_fixture(gpu_available, mode):
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
    al = snapgpu.BaseAligner(idx)
    seeds = open(os.path.join(G, "lookup_seeds.txt")).read().split()
    want = open(os.path.join(G, "expected_lookups.tsv")).read().splitlines()
    out, lines = al.lookup_seeds(seeds, mode=mode)
    got = _fixture_rows(out)
    bad = [(s, g, w) for s, g, w in zip(seeds, got, want) if g != w]
    assert len(got) == len(want) and not bad, bad[:3]
    assert lines.min() >= 1


@pytest.mark.gpu
def test_gpu_lookups_on_reference_built_index(gpu_available, tmp_path):
    with tarfile.open(os.path.join(G, "small_ref_index.tar.gz"), "r:gz") as t:
        t.extractall(tmp_path)
    idx = snapgpu.GenomeIndex.load(str(tmp_path))
    al = snapgpu.BaseAligner(idx)
    seeds = open(os.path.join(G, "lookup_seeds.txt")).read().split()
    want = open(os.path.join(G, "expected_lookups.tsv")).read().splitlines()
    for mode in (0, 1, 2):
        got = _fixture_rows(al.lookup_seeds(seeds, mode=mode)[0])
        assert got == want, mode
    bi = al.bucket_info()
    assert 0 < bi["nKeys"] <= idx.info()["totalUsedSlots"] and bi["bytes"] == 64 * bi["nBuckets"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed_len", [16, 20, 25])
def test_gpu_lookups_match_host(gpu_available, small_world, seed_len):
    g = small_world["genome"].bases()
    # GenomeIndex.build takes ownership of its genome: the other seed lengths index a fresh copy
    idx = small_world["index"] if seed_len == 20 else snapgpu.GenomeIndex.build(
        snapgpu.Genome.synthetic(1_000_000, seed=2121, n_contigs=3, n_repeat_families=60), seed_len, 8)
    al = snapgpu.BaseAligner(idx)
    seeds = _seed_set(g, seed_len, 6000, 3000)
    want = _host_rows(idx, seeds)
    for mode in (0, 1, 2):
        out, lines = al.lookup_seeds(seeds, mode=mode)
        got = _fixture_rows(out)
        bad = [i for i in range(len(seeds)) if got[i] != want[i]]
        assert not bad, (mode, [(seeds[i], got[i], want[i]) for i in bad[:3]])
        if mode == 0:
            lines0 = lines
        else:
            assert np.array_equal(lines, lines0)   # every form counts the buckets a sequential lookup loads
    assert max(int(w.split("\t")[0]) for w in want) > 1   # overflow lists are in the set
    bi = al.bucket_info()
    info = idx.info()
    assert bi["nSlots"] == info["totalHashSlots"] and bi["nKeys"] == info["totalUsedSlots"]
    assert bi["nBuckets"] >= (bi["nKeys"] + 1) // 2 and bi["bytes"] == 64 * bi["nBuckets"]
    assert bi["nOverflowBuckets"] < 0.2 * bi["nBuckets"]
    assert float(lines0.mean()) < 1.2, float(lines0.mean())   # one line per lookup in the common case


@pytest.mark.gpu
def test_gpu_lookups_saturated_counts(gpu_available, tmp_path):
    """Seeds of a 200 kb tandem array occur ~40,000 times: past the entry's 15-bit count field
    (BK_CSAT), so the device re-reads the count from the overflow list."""
    rng = np.random.default_rng(11)
    body = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 100_000)].tobytes() + b"AACGT" * 40_000
    fa = tmp_path / "tandem.fa"
    fa.write_bytes(b">tandem\n" + b"\n".join(body[i:i + 80] for i in range(0, len(body), 80)) + b"\n")
    g = snapgpu.Genome.from_fasta(str(fa), 500)
    gb = g.bases()
    idx = snapgpu.GenomeIndex.build(g, 20, 8)
    al = snapgpu.BaseAligner(idx)
    seeds = [(b"AACGT" * 5)[k:k + 20].decode() for k in range(5)] + _seed_set(gb, 20, 500, 200)
    want = _host_rows(idx, seeds)
    assert max(int(w.split("\t")[0]) for w in want[:5]) > 0x7fff
    for mode in (0, 1, 2):
        assert _fixture_rows(al.lookup_seeds(seeds, mode=mode)[0]) == want, mode


@pytest.mark.gpu
def test_gpu_lookup_rejects_non_acgt(gpu_available, small_world):
    al = snapgpu.BaseAligner(small_world["index"])
    with pytest.raises(snapgpu.SnapGpuError):
        al.lookup_seeds(["ACGTNACGTACGTACGTACG"])


@pytest.mark.gpu
def test_gpu_bucket_layout_is_deterministic(gpu_available, small_world):
    """Two aligners build the image independently (racing atomic placements): the layout -- and so
    the lines every lookup loads, snapgpu_result_t::nProbes -- is the same."""
    idx = small_world["index"]
    seeds = _seed_set(small_world["genome"].bases(), 20, 4000, 2000, seed=9)
    a, b = snapgpu.BaseAligner(idx), snapgpu.BaseAligner(idx)
    la, lb = a.lookup_seeds(seeds, mode=0)[1], b.lookup_seeds(seeds, mode=0)[1]
    assert np.array_equal(la, lb)
    assert a.bucket_info()["nOverflowBuckets"] == b.bucket_info()["nOverflowBuckets"]
    reads = small_world["reads"]
    assert np.array_equal(a.AlignReads(reads)["nProbes"], b.AlignReads(reads)["nProbes"])

"""CPU tests of the C ABI boundary (include/snapgpu.h): the library loads, exports
every declared entry point, and the host-side (no GPU) calls behave."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import snapgpu
from snapgpu import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "snapgpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(snapgpu_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_ffi.LIB_PATH)
    decl = declared_functions()
    assert len(decl) >= 35
    missing = [f for f in decl if not hasattr(lib, f)]
    assert not missing, missing
    # and the ctypes layer binds exactly the header's functions
    assert sorted(_ffi.EXPORTED_SYMBOLS) == decl


def test_struct_layout():
    assert C.sizeof(_ffi.Result) == 64
    assert snapgpu.RESULT_DTYPE.itemsize == 64
    assert _ffi.lib().snapgpu_abi_version() == 1


def test_default_params_match_reference_defaults():
    p = snapgpu.default_params()   # AlignerOptions.cpp:33-85 / SingleAligner.cpp:167-179
    assert (p.maxHitsToConsider, p.maxK, p.maxReadSize, p.maxSeedsToUse, p.extraSearchDepth) == (300, 14, 500, 25, 2)


def test_genome_fasta_semantics(tmp_path):
    fa = tmp_path / "g.fa"
    fa.write_text(">chrA some description\nACGTNNacgt\nRYKM\n>chrB\tx\nGGGG\n")
    g = snapgpu.Genome.from_fasta(fa, chromosome_padding=10)
    # FASTA.cpp:67-125: padding before each contig and at the end, upper-case, N -> n
    assert g.bases(0, g.n_bases) == b"n" * 10 + b"ACGTnnACGTRYKM" + b"n" * 10 + b"GGGG" + b"n" * 10
    assert g.pieces == [("chrA", 10), ("chrB", 34)]


def test_index_save_load_roundtrip(tmp_path):
    g = snapgpu.Genome.synthetic(200_000, seed=5, n_contigs=2, n_repeat_families=20)
    idx = snapgpu.GenomeIndex.build(g, 20, 2)
    idx.save(tmp_path / "idx")
    assert sorted(os.listdir(tmp_path / "idx")) == ["Genome", "GenomeIndex", "GenomeIndexHash", "OverflowTable"]
    idx2 = snapgpu.GenomeIndex.load(tmp_path / "idx")
    i1, i2 = idx.info(), idx2.info()
    assert i1 == i2
    v1, v2 = idx.view(), idx2.view()
    assert C.string_at(v1.genome, i1["nBases"]) == C.string_at(v2.genome, i2["nBases"])
    rng = np.random.default_rng(1)
    for p in rng.integers(1000, i1["nBases"] - 1000, 300):
        s = idx.genome_bases(int(p), 20).decode()
        if set(s) <= set("ACGT"):
            assert idx.lookupSeed(s) == idx2.lookupSeed(s)


def test_index_semantics_brute_force():
    """lookupSeed == every offset whose 20 bases equal the seed (FORWARD) or its
    reverse complement (RC), overflow lists descending (GenomeIndex.cpp:546-619)."""
    g = snapgpu.Genome.synthetic(60_000, seed=11, n_contigs=2, n_repeat_families=8, max_divergence=0.02)
    text = g.bases(0, g.n_bases).decode()
    idx = snapgpu.GenomeIndex.build(g, 20, 2)
    nb = len(text)
    occ = {}
    for p in range(0, nb - 21):
        s = text[p:p + 20]
        if set(s) <= set("ACGT"):
            occ.setdefault(s, []).append(p)
    comp = str.maketrans("ACGT", "TGCA")
    rng = np.random.default_rng(2)
    keys = list(occ)
    for j in rng.integers(0, len(keys), 400):
        s = keys[int(j)]
        f, r, _ = idx.lookupSeed(s)
        assert f == sorted(occ[s], reverse=True)
        rc = s.translate(comp)[::-1]
        assert r == sorted(occ.get(rc, []), reverse=True)


def test_reads_generator_deterministic():
    g1 = snapgpu.Genome.synthetic(300_000, seed=1, n_contigs=2)
    g2 = snapgpu.Genome.synthetic(300_000, seed=1, n_contigs=2)
    assert g1.bases() == g2.bases()
    r1 = snapgpu.Reads.synthetic(g1, 500, seed=3)
    r2 = snapgpu.Reads.synthetic(g2, 500, seed=3)
    assert all(r1.get(i) == r2.get(i) for i in range(500))


def test_aligner_fails_loudly_without_gpu():
    if snapgpu.device_count() > 0:
        pytest.skip("GPU present")
    g = snapgpu.Genome.synthetic(100_000, seed=1)
    idx = snapgpu.GenomeIndex.build(g, 20, 1)
    with pytest.raises(snapgpu.SnapGpuError):
        snapgpu.BaseAligner(idx)


def test_plain_c_caller(tmp_path):
    """tests/c/abi_smoke.c: the header compiles as C99 (-Wall -Wextra -pedantic) and a C
    program linked against the library runs the host-side entry points."""
    import subprocess
    exe = tmp_path / "abi_smoke"
    libdir = os.path.dirname(_ffi.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_smoke.c"), "-o", str(exe), "-L", libdir, "-lsnapgpu",
                    "-Wl,-rpath," + libdir], check=True)
    env = dict(os.environ)
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok 1" in out.stdout

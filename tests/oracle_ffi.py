"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")

_orc = None


def oracle_lib():
    global _orc
    if _orc is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "oracle", "Makefile")], check=True, cwd=ROOT)
        import snapgpu._ffi as F
        o = C.CDLL(ORACLE_SO)
        o.oracle_align_batch.argtypes = [C.POINTER(F.IndexView), C.POINTER(F.AlignerParams), C.c_void_p, C.c_void_p,
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_uint64,
                                         C.c_void_p, C.c_int]
        o.oracle_align_batch.restype = C.c_int
        o.oracle_align_batch_ex.argtypes = [C.POINTER(F.IndexView), C.POINTER(F.AlignerParams), C.c_void_p,
                                            C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_uint64,
                                            C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        o.oracle_align_batch_ex.restype = C.c_int
        o.oracle_lv.argtypes = [C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int, C.c_int,
                                C.POINTER(C.c_double), C.POINTER(C.c_int)]
        o.oracle_lv.restype = C.c_int
        o.oracle_cigar.argtypes = [C.POINTER(F.IndexView), C.c_uint32, C.c_char_p, C.c_int, C.c_int,
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
        o.oracle_cigar.restype = C.c_int
        o.oracle_paired_batch.argtypes = [C.POINTER(F.IndexView), C.POINTER(F.PairedParams)] + [C.c_void_p] * 8 + \
            [C.c_uint64, C.c_int, C.c_void_p, C.c_int]
        o.oracle_paired_batch.restype = C.c_int
        o.oracle_characterize_seeds.argtypes = [C.POINTER(F.IndexView), C.c_uint, C.c_uint, C.c_uint, C.c_int,
                                                C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_uint64]
        o.oracle_characterize_seeds.restype = C.c_int
        o.oracle_compute_mapq.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int]
        o.oracle_compute_mapq.restype = C.c_int
        _orc = o
    return _orc


def oracle_align(index, reads, params, n_threads=8):
    """CPU restatement of BaseAligner::AlignRead over the same index and reads."""
    import snapgpu
    from snapgpu import _ffi as F
    v = index.view()
    n = reads.n
    out = np.zeros(max(1, n), dtype=snapgpu.RESULT_DTYPE)
    r = reads._p.contents
    rc = oracle_lib().oracle_align_batch(C.byref(v), C.byref(params), r.bases, r.quals, r.offsets, r.lengths, n,
                                         out.ctypes.data, n_threads)
    assert rc == 0
    return out[:n]


def oracle_paired(index, reads0, reads1, params, chimeric=True, n_threads=8):
    """CPU restatement of ChimericPairedEndAligner::align (or IntersectingPairedEndAligner::align
    alone) for every pair (reads0[i], reads1[i])."""
    import snapgpu
    assert reads0.n == reads1.n
    v = index.view()
    n = reads0.n
    out = np.zeros(max(1, n), dtype=snapgpu.PAIR_RESULT_DTYPE)
    a, b = reads0._p.contents, reads1._p.contents
    rc = oracle_lib().oracle_paired_batch(C.byref(v), C.byref(params), a.bases, a.quals, C.cast(a.offsets, C.c_void_p),
                                          C.cast(a.lengths, C.c_void_p), b.bases, b.quals,
                                          C.cast(b.offsets, C.c_void_p), C.cast(b.lengths, C.c_void_p), n,
                                          int(chimeric), out.ctypes.data, n_threads)
    assert rc == 0
    return out[:n]


def oracle_charseeds(index, reads, maxHits=300, maxK=15, numSeeds=12, explore=0):
    """CPU restatement of BaseAligner::CharacterizeSeeds -> (start, nForward, runs) as
    snapgpu.characterize_seeds returns them (flags aside)."""
    import snapgpu
    v = index.view()
    n = reads.n
    r = reads._p.contents
    cap = max(1, n) * (numSeeds + 1) * maxHits
    start = np.zeros(n + 1, dtype=np.uint64)
    nfwd = np.zeros(max(1, n), dtype=np.uint32)
    runs = np.zeros(cap, dtype=snapgpu.SEED_RUN_DTYPE)
    rc = oracle_lib().oracle_characterize_seeds(C.byref(v), maxHits, maxK, numSeeds, explore, r.bases,
                                                C.cast(r.offsets, C.c_void_p), C.cast(r.lengths, C.c_void_p), n,
                                                start.ctypes.data, nfwd.ctypes.data, runs.ctypes.data, cap)
    assert rc == 0
    return start, nfwd[:n], runs[:int(start[n])]


def parse_charseeds(text):
    """ref_harness_rna charseeds lines -> list per read of (nF, nRC, [(dir, loc, min, max, count), ...])."""
    out = []
    for line in text.splitlines():
        f = line.split("\t")
        runs = []
        for d, col in ((0, f[3]), (1, f[4])):
            body = col.split(":", 1)[1] if ":" in col else ""
            for item in filter(None, body.split(",")):
                loc, mn, mx, cnt = (int(x) for x in item.split(":"))
                runs.append((d, loc, mn, mx, cnt))
        out.append((int(f[1]), int(f[2]), runs))
    return out


def runs_as_lists(start, nfwd, runs):
    """(start, nForward, runs) -> the parse_charseeds form, for comparisons."""
    out = []
    for i in range(len(start) - 1):
        rs = runs[int(start[i]):int(start[i + 1])]
        lst = [(int(x["direction"]), int(x["location"]), int(x["minOffset"]), int(x["maxOffset"]), int(x["count"]))
               for x in rs]
        out.append((int(nfwd[i]), len(lst) - int(nfwd[i]), lst))
    return out


PAIR_FIELDS = ("status", "location", "direction", "score", "mapq")


def paired_tsv_rows(res, chimeric=True):
    """The ref_harness paired columns of one aligner (canonical text per pair)."""
    rows = []
    for r in res:
        f = [int(r["status"][0]), int(r["status"][1]), int(r["location"][0]), int(r["location"][1]),
             int(r["direction"][0]), int(r["direction"][1]), int(r["score"][0]), int(r["score"][1]),
             int(r["mapq"][0]), int(r["mapq"][1])]
        if chimeric:
            f += [int(r["fromAlignTogether"]), int(r["alignedAsPair"]), int(r["nLocationsScored"]) + int(r["nSingleScored"])]
        else:
            f += [int(r["nLocationsScored"])]
        rows.append("\t".join(map(str, f)))
    return rows


def ref_paired_rows(path):
    """Split ref_harness paired output into (intersecting rows, chimeric rows)."""
    inter, chim = [], []
    for line in open(path):
        c = line.rstrip("\n").split("\t")
        inter.append("\t".join(c[1:12]))
        chim.append("\t".join(c[12:25]))
    return inter, chim


def oracle_align_ex(index, reads, params, search=None, max_hits_to_get=0, n_threads=8):
    """The richer AlignRead (BaseAligner.h:73-86): per-read search windows (an (n, 3)
    array of radius, location, direction, or None) and multi-hit export.
    -> (results, multiHitsFound int32[n], multiHits MULTI_HIT_DTYPE[n, max_hits_to_get])."""
    import snapgpu
    v = index.view()
    n = reads.n
    out = np.zeros(max(1, n), dtype=snapgpu.RESULT_DTYPE)
    found = np.zeros(max(1, n), dtype=np.int32)
    hits = np.zeros((max(1, n), max(1, max_hits_to_get)), dtype=snapgpu.MULTI_HIT_DTYPE)
    srch = snapgpu.search_array(search, n)
    r = reads._p.contents
    rc = oracle_lib().oracle_align_batch_ex(C.byref(v), C.byref(params), r.bases, r.quals, r.offsets, r.lengths, n,
                                            None if srch is None else srch.ctypes.data, max_hits_to_get,
                                            out.ctypes.data, found.ctypes.data, hits.ctypes.data, n_threads)
    assert rc == 0
    return out[:n], found[:n], hits[:n, :max_hits_to_get]


def canonical_tsv_ex(res, found, hits):
    """canonical_tsv + nFound + "loc:dir:score,..." (the ref_harness alignx form)."""
    base = canonical_tsv(res).splitlines()
    lines = []
    for i, b in enumerate(base):
        f = int(found[i])
        h = ",".join(f"{int(x['location'])}:{int(x['direction'])}:{int(x['score'])}" for x in hits[i, :max(f, 0)])
        lines.append(f"{b}\t{f}\t{h or '-'}")
    return "\n".join(lines) + "\n"


def oracle_lv(direction, text, pattern, quals, k):
    """LandauVishkin<direction>::computeEditDistance; text padded with 'n' as the
    reference harness does (oracle/ref_harness.cpp mode_lv)."""
    t = text.encode() if isinstance(text, str) else bytes(text)
    p = pattern.encode() if isinstance(pattern, str) else bytes(pattern)
    q = quals.encode() if isinstance(quals, str) else bytes(quals)
    tbuf = C.create_string_buffer(b"n" * 64 + t + b"n" * 64)
    pbuf = C.create_string_buffer(p + b"\0" * 16)
    qbuf = C.create_string_buffer(q.ljust(len(p), b"!") + b"\0" * 16)
    prob = C.c_double()
    net = C.c_int()
    base = C.addressof(tbuf) + 64 + (0 if direction > 0 else len(t))
    e = oracle_lib().oracle_lv(direction, C.c_char_p(base), len(t), pbuf, qbuf, len(p), k, C.byref(prob),
                               C.byref(net))
    return e, net.value, prob.value


# Every record field, bitwise -- except nProbes: on the device it counts the 64-B lines of the
# seed tables' bucket image a read's lookups loaded (include/snapgpu.h), in the oracle the
# reference's SNAPHashTable probes; neither is an AlignRead output.
COMPARE_FIELDS = ("result", "location", "direction", "score", "mapq", "nLookups", "nLocationsScored",
                  "popularSeedsSkipped", "nHitsIgnored", "nHitWords", "nOverflowLists", "nElements",
                  "probabilityOfAllCandidates", "probabilityOfBestCandidate")


NUL_FLAG = 0x20   # SNAPGPU_FLAG_NUL_BYTE: a read holds a 0x00 byte (a corrupted upload)


def assert_no_corrupt_reads(res):
    """No record of a GPU result array may carry SNAPGPU_FLAG_NUL_BYTE: every test input comes from
    FASTQ or the synthetic generators, neither of which produces a 0x00 byte inside a read, so a
    flagged record means the device saw bytes the host did not send."""
    if "flags" in res.dtype.names:
        nul = np.nonzero(res["flags"] & NUL_FLAG)[0]
        assert len(nul) == 0, f"{len(nul)} reads arrived on the device with 0x00 bytes, first {nul[:5]}"


def mismatches(a, b, fields=COMPARE_FIELDS):
    """Indices where two result arrays differ in any field (doubles compared bitwise).  Both arrays
    are also checked for records of corrupted uploads (assert_no_corrupt_reads)."""
    assert_no_corrupt_reads(a)
    assert_no_corrupt_reads(b)
    bad = np.zeros(len(a), dtype=bool)
    for f in fields:
        if a.dtype[f].kind == "f":
            bad |= a[f].view(np.uint64) != b[f].view(np.uint64)
        else:
            bad |= a[f] != b[f]
    return np.nonzero(bad)[0]


def canonical_tsv(res):
    """Canonical text form of results (golden fixtures / digests): doubles as IEEE bits."""
    pa = res["probabilityOfAllCandidates"].view(np.uint64)
    pb = res["probabilityOfBestCandidate"].view(np.uint64)
    lines = []
    for i in range(len(res)):
        r = res[i]
        lines.append(f"{i}\t{r['result']}\t{r['location']}\t{r['direction']}\t{r['score']}\t{r['mapq']}\t"
                     f"{r['nLookups']}\t{r['nLocationsScored']}\t{r['popularSeedsSkipped']}\t"
                     f"{int(pa[i]):016x}\t{int(pb[i]):016x}")
    return "\n".join(lines) + "\n"


_UPPER = bytes(c - 32 if 97 <= c <= 122 else c for c in range(256))      # Tables.cpp:74-80
_COMP = bytearray(256)                                                     # Tables.cpp:22-30
for a, b in zip(b"ACGTNn", b"TGCANn"):
    _COMP[a] = b
_COMP = bytes(_COMP)


def sam_pattern(read, direction):
    """The read as getSAMData hands it to computeCigarString (SAM.cpp:866-883)."""
    r = (read.encode() if isinstance(read, str) else bytes(read)).translate(_UPPER)
    return r.translate(_COMP)[::-1] if direction else r


def oracle_cigars(index, reads_bases, locations, directions, use_m):
    """CPU restatement of computeCigarString -> list of (editDistance, cigar string)."""
    import snapgpu
    v = index.view()
    ops = (C.c_uint32 * 64)()
    nops = C.c_int()
    out = []
    for b, loc, d in zip(reads_bases, locations, directions):
        p = sam_pattern(b, d)
        if int(loc) == 0xFFFFFFFF:
            out.append((-1, "*"))
            continue
        ed = oracle_lib().oracle_cigar(C.byref(v), int(loc), p + b"\0" * 16, len(p), int(use_m), ops,
                                       C.byref(nops))
        s = "*" if ed < 0 else "".join(f"{ops[k] >> 4}{snapgpu.CIGAR_OPS[ops[k] & 15]}" for k in range(nops.value))
        out.append((ed, s))
    return out

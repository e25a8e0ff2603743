"""snapgpu -- MI355X-native drop-in for SNAP's BaseAligner hot path.

Python mirror of the reference's C++ surface (SNAPLib/Aligner.h:54-80,
SNAPLib/BaseAligner.h:44-142, SNAPLib/GenomeIndex.h) over the C ABI of
include/snapgpu.h.  Every call goes to the native library: genome/index work is
host C++, alignment is HIP on gfx950.  There is no CPU fallback -- creating a
BaseAligner without a GPU raises.
"""
import ctypes as C
import time

import numpy as np

from . import _ffi
from ._ffi import lib, last_error

NotFound, SingleHit, MultipleHits, UnknownAlignment = 0, 1, 2, 3   # Read.h:41
FORWARD, RC = 0, 1                                                  # directions.h:26-35
InvalidGenomeLocation = 0xFFFFFFFF                                  # Genome.h:29
UnusedScoreValue = 0xFFFF                                           # BaseAligner.h:261

FLAG_READ_TOO_LONG = 0x01
FLAG_MAPQ_FIXED = 0x02
FLAG_DEFERRED = 0x04
FLAG_BYTE_PATH = 0x10
FLAG_TOO_MANY_NS = 0x08
FLAG_NUL_BYTE = 0x20     # a 0x00 byte inside the read: a corrupted upload (no reader produces one)

RESULT_DTYPE = np.dtype([
    ("location", "<u4"), ("score", "<i4"), ("mapq", "<i4"), ("result", "u1"), ("direction", "u1"),
    ("flags", "u1"), ("reserved", "u1"), ("nLookups", "<u4"), ("nLocationsScored", "<u4"),
    ("popularSeedsSkipped", "<u2"), ("nHitsIgnored", "<u2"), ("nProbes", "<u4"), ("nHitWords", "<u4"),
    ("nOverflowLists", "<u4"), ("nElements", "<u4"), ("reserved2", "<u4"),
    ("probabilityOfAllCandidates", "<f8"), ("probabilityOfBestCandidate", "<f8"),
])
assert RESULT_DTYPE.itemsize == C.sizeof(_ffi.Result)

# snapgpu_pair_result_t (include/snapgpu.h): PairedAlignmentResult (PairedEndAligner.h:31-55)
PAIR_RESULT_DTYPE = np.dtype([
    ("location", "<u4", (2,)), ("score", "<i4", (2,)), ("mapq", "<i4", (2,)), ("status", "u1", (2,)),
    ("direction", "u1", (2,)), ("fromAlignTogether", "u1"), ("alignedAsPair", "u1"), ("flags", "<u2"),
    ("nLocationsScored", "<u4"), ("nSingleScored", "<u4"), ("popularSeedsSkipped", "<u4"), ("writtenBy", "<u4"),
    ("probabilityOfAllPairs", "<f8"), ("probabilityOfBestPair", "<f8"),
])
assert PAIR_RESULT_DTYPE.itemsize == 64
PFLAG_POOL_EXHAUSTED, PFLAG_READ_TOO_LONG, PFLAG_DEFERRED, PFLAG_MAPQ_FIXED = 0x01, 0x02, 0x04, 0x08
PFLAG_NUL_BYTE = 0x10

# snapgpu_search_t / snapgpu_multi_hit_t (include/snapgpu.h)
SEARCH_DTYPE = np.dtype([("searchRadius", "<u4"), ("searchLocation", "<u4"), ("searchDirection", "<u4"),
                         ("reserved", "<u4")])
MULTI_HIT_DTYPE = np.dtype([("location", "<u4"), ("direction", "u1"), ("score", "u1"), ("reserved", "<u2")])
MAX_MULTI_HITS_TO_GET = 512   # BaseAligner.h:149


def search_array(search, n):
    """None, a SEARCH_DTYPE array, or an (n, 3) array-like of (radius, location, direction)."""
    if search is None:
        return None
    s = np.asarray(search)
    if s.dtype != SEARCH_DTYPE:
        a = np.asarray(search, dtype=np.uint64).reshape(-1, 3)
        s = np.zeros(len(a), dtype=SEARCH_DTYPE)
        s["searchRadius"], s["searchLocation"], s["searchDirection"] = a[:, 0], a[:, 1], a[:, 2]
    if len(s) != n:
        raise ValueError(f"search has {len(s)} entries for {n} reads")
    return np.ascontiguousarray(s)


class SnapGpuError(RuntimeError):
    pass


_PTR_CALLS = ("genome_from_fasta", "genome_synthetic", "index_build", "index_load", "index_attach", "gtf_load",
              "reads_synthetic",
              "reads_from_fastq", "reads_from_arrays", "aligner_create", "reads_upload", "paired_aligner_create",
              "contaminants_create")


def _check(value, what):
    """Pointer-returning calls fail on NULL; int-returning calls on a non-zero code."""
    if what in _PTR_CALLS:
        if not value:
            raise SnapGpuError(f"{what} failed: {last_error()}")
        return value
    if value != 0:
        raise SnapGpuError(f"{what} failed ({value}): {last_error()}")
    return value


def device_cu_count(device=0):
    return lib().snapgpu_device_cu_count(device)


def device_count():
    return lib().snapgpu_device_count()


def host_threads():
    """This rank's host thread budget (snapgpu_host_threads): affinity mask capped by the cgroup
    CPU quota, divided by LOCAL_WORLD_SIZE; SNAPGPU_HOST_THREADS overrides."""
    return lib().snapgpu_host_threads()


class Genome:
    """Whole-genome byte string with contig padding (SNAPLib/Genome.h)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_fasta(cls, path, chromosome_padding=500):
        return cls(_check(lib().snapgpu_genome_from_fasta(str(path).encode(), chromosome_padding), "genome_from_fasta"))

    @classmethod
    def synthetic(cls, total_bases, seed=2121, n_contigs=1, n_repeat_families=200, repeat_fraction=0.45,
                  max_divergence=0.15, n_run_fraction=0.002, chromosome_padding=500):
        p = _ffi.SynthGenomeParams(seed=seed, totalBases=total_bases, nContigs=n_contigs,
                                   nRepeatFamilies=n_repeat_families, repeatFraction=repeat_fraction,
                                   maxDivergence=max_divergence, nRunFraction=n_run_fraction,
                                   chromosomePadding=chromosome_padding)
        return cls(_check(lib().snapgpu_genome_synthetic(C.byref(p)), "genome_synthetic"))

    def write_fasta(self, path):
        _check(lib().snapgpu_genome_write_fasta(self._h, str(path).encode()), "write_fasta")

    @property
    def n_bases(self):
        return lib().snapgpu_genome_nbases(self._h)

    def bases(self, start=0, length=None):
        n = self.n_bases
        if length is None:
            length = n - start
        return C.string_at(lib().snapgpu_genome_bases(self._h) + start, length)

    @property
    def pieces(self):
        L = lib()
        return [(L.snapgpu_genome_piece_name(self._h, i).decode(), L.snapgpu_genome_piece_offset(self._h, i))
                for i in range(L.snapgpu_genome_npieces(self._h))]

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_genome_free(self._h)
            self._h = None


class GenomeIndex:
    """Seed index with GenomeIndex::lookupSeed semantics (SNAPLib/GenomeIndex.cpp:971-1086)."""

    def __init__(self, handle, genome_keepalive=None):
        self._h = handle

    @classmethod
    def build(cls, genome, seed_len=20, n_threads=0, slack=0.3):
        """GenomeIndex::BuildIndexToDirectory semantics with the reference's table sizing
        (slack as `snap-rna index -h`); takes ownership of the genome."""
        h = genome._h
        genome._h = None          # ownership moves to the index
        return cls(_check(lib().snapgpu_index_build_ex(h, seed_len, n_threads, float(slack)), "index_build"))

    @classmethod
    def load(cls, directory):
        return cls(_check(lib().snapgpu_index_load(str(directory).encode()), "index_load"))

    def share(self, path):
        """Write the flat shared form (one file, e.g. under /dev/shm) for snapgpu_index_attach."""
        _check(lib().snapgpu_index_share(self._h, str(path).encode()), "index_share")

    @classmethod
    def attach(cls, path):
        """Map a shared index read-only (no private copy of the tables)."""
        return cls(_check(lib().snapgpu_index_attach(str(path).encode()), "index_attach"))

    def genome_handle(self):
        """The owned genome (a raw handle for Reads.synthetic; valid while the index lives)."""
        return lib().snapgpu_index_genome(self._h)

    def save(self, directory):
        _check(lib().snapgpu_index_save(self._h, str(directory).encode()), "index_save")

    def info(self):
        i = _ffi.IndexInfo()
        _check(lib().snapgpu_index_get_info(self._h, C.byref(i)), "index_info")
        return {f: getattr(i, f) for f, _ in i._fields_}

    def view(self):
        v = _ffi.IndexView()
        _check(lib().snapgpu_index_get_view(self._h, C.byref(v)), "index_view")
        return v

    def getSeedLength(self):
        return self.info()["seedLen"]

    def genome_bases(self, start, length):
        v = self.view()
        return C.string_at(v.genome + start, length)

    def lookupSeed(self, seed, cap=1 << 20):
        """-> (hits, rcHits): lists of genome offsets (overflow lists descending)."""
        n = (C.c_uint32 * 2)()
        buf = max(1, cap)
        f = (C.c_uint32 * buf)()
        r = (C.c_uint32 * buf)()
        rc = lib().snapgpu_index_lookup(self._h, seed.encode() if isinstance(seed, str) else seed, n, f, r, buf)
        if rc != 0:
            raise SnapGpuError(f"lookup failed: {last_error()}")
        return list(f[:min(n[0], buf)]), list(r[:min(n[1], buf)]), (n[0], n[1])

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_index_free(self._h)
            self._h = None


class Reads:
    """A host batch of reads (bases + Phred+33 qualities), Read.h:289-328 contract."""

    def __init__(self, ptr):
        self._p = ptr

    @classmethod
    def synthetic(cls, genome, n_reads, seed=99, read_length=100, quality_char="2", base_error_rate=0.02,
                  mutation_rate=0.001, indel_fraction=0.15, indel_extend=0.3, random_read_fraction=0.0):
        p = _ffi.SynthReadsParams(seed=seed, nReads=n_reads, readLength=read_length,
                                  qualityChar=ord(quality_char), baseErrorRate=base_error_rate,
                                  mutationRate=mutation_rate, indelFraction=indel_fraction,
                                  indelExtend=indel_extend, randomReadFraction=random_read_fraction)
        g = genome._h if isinstance(genome, Genome) else genome
        return cls(_check(lib().snapgpu_reads_synthetic(g, C.byref(p)), "reads_synthetic"))

    @classmethod
    def synthetic_pairs(cls, genome, n_pairs, seed=99, read_length=101, insert_mean=500, insert_sd=50,
                        quality_char="2", base_error_rate=0.02, mutation_rate=0.001, indel_fraction=0.15,
                        indel_extend=0.3):
        """wgsim-like pairs (snapgpu_reads_synthetic_pairs) -> (reads0, reads1)."""
        p = _ffi.SynthReadsParams(seed=seed, nReads=n_pairs, readLength=read_length,
                                  qualityChar=ord(quality_char), baseErrorRate=base_error_rate,
                                  mutationRate=mutation_rate, indelFraction=indel_fraction,
                                  indelExtend=indel_extend, randomReadFraction=0.0)
        g = genome._h if isinstance(genome, Genome) else genome
        a, b = C.POINTER(_ffi.Reads)(), C.POINTER(_ffi.Reads)()
        _check(lib().snapgpu_reads_synthetic_pairs(g, C.byref(p), insert_mean, insert_sd, C.byref(a), C.byref(b)),
               "reads_synthetic_pairs")
        return cls(a), cls(b)

    @classmethod
    def from_fastq(cls, path):
        return cls(_check(lib().snapgpu_reads_from_fastq(str(path).encode()), "reads_from_fastq"))

    @classmethod
    def from_list(cls, reads):
        """reads: iterable of (bases, quals) str/bytes pairs."""
        bases, quals, offs, lens = bytearray(), bytearray(), [], []
        for b, q in reads:
            b = b.encode() if isinstance(b, str) else bytes(b)
            q = q.encode() if isinstance(q, str) else bytes(q)
            if len(q) < len(b):
                q = q + b"!" * (len(b) - len(q))
            offs.append(len(bases))
            lens.append(len(b))
            bases += b
            quals += q[:len(b)]
        n = len(lens)
        bases += b"\0" * 16
        quals += b"\0" * 16
        o = (C.c_uint64 * max(1, n))(*offs)
        l = (C.c_uint32 * max(1, n))(*lens)
        return cls(_check(lib().snapgpu_reads_from_arrays(n, bytes(bases), bytes(quals), o, l), "reads_from_arrays"))

    def slice(self, start, count):
        """A copy of reads [start, start + count) as a new batch."""
        r = self._p.contents
        count = max(0, min(count, r.n - start))
        offs = C.cast(C.addressof(r.offsets.contents) + 8 * start, C.POINTER(C.c_uint64))
        lens = C.cast(C.addressof(r.lengths.contents) + 4 * start, C.POINTER(C.c_uint32))
        return Reads(_check(lib().snapgpu_reads_from_arrays(count, C.cast(r.bases, C.c_char_p),
                                                            C.cast(r.quals, C.c_char_p), offs, lens),
                            "reads_from_arrays"))

    @property
    def n(self):
        return self._p.contents.n

    def __len__(self):
        return self.n

    def lengths(self):
        """Read lengths as a uint32 array (a copy)."""
        r = self._p.contents
        return np.ctypeslib.as_array(r.lengths, shape=(r.n,)).copy() if r.n else np.zeros(0, np.uint32)

    def get(self, i):
        r = self._p.contents
        o, l = r.offsets[i], r.lengths[i]
        return C.string_at(r.bases + o, l), C.string_at(r.quals + o, l)

    def ids(self):
        """Read ids (FASTQ header without '@'), or None when the batch has none."""
        r = self._p.contents
        if not r.ids:
            return None
        return [C.string_at(r.ids + r.idOffsets[i], r.idLengths[i]) for i in range(r.n)]

    def truth(self):
        r = self._p.contents
        if not r.truthLocation:
            return None
        n = r.n
        loc = np.ctypeslib.as_array(r.truthLocation, shape=(n,)).copy()
        d = np.ctypeslib.as_array(r.truthDirection, shape=(n,)).copy()
        return loc, d

    def clip(self, clipping=3):
        """Read::clip (Read.h:357-404) on every read, in place (the FASTQ reader's step,
        FASTQ.cpp:250; 0 none, 1 front, 2 back, 3 front and back = the reference default).
        -> (frontClipped, unclippedLength) uint32 arrays for sam_format(clip=...)."""
        n = self.n
        front = np.zeros(max(1, n), dtype=np.uint32)
        full = np.zeros(max(1, n), dtype=np.uint32)
        _check(lib().snapgpu_reads_clip(self._p, int(clipping), front.ctypes.data, full.ctypes.data), "reads_clip")
        return front[:n], full[:n]

    def write_fastq(self, path):
        _check(lib().snapgpu_reads_write_fastq(self._p, str(path).encode()), "write_fastq")

    def __del__(self):
        if getattr(self, "_p", None):
            lib().snapgpu_reads_free(self._p)
            self._p = None


def default_params():
    p = _ffi.AlignerParams()
    lib().snapgpu_aligner_params_default(C.byref(p))
    return p


class BaseAligner:
    """GPU BaseAligner (SNAPLib/BaseAligner.h:41-142).

    Constructor arguments follow BaseAligner::BaseAligner (BaseAligner.h:44-55);
    AlignRead follows BaseAligner::AlignRead (BaseAligner.cpp:196-200); AlignReads
    is the batched form the GPU is built for.
    """

    def __init__(self, index, maxHitsToConsider=300, maxK=14, maxReadSize=500, maxSeedsToUse=25,
                 maxSeedCoverage=0.0, extraSearchDepth=2, explorePopularSeeds=False, stopOnFirstHit=False,
                 device=0):
        self.index = index
        self.params = _ffi.AlignerParams(maxHitsToConsider=maxHitsToConsider, maxK=maxK, maxReadSize=maxReadSize,
                                         maxSeedsToUse=maxSeedsToUse, maxSeedCoverage=maxSeedCoverage,
                                         extraSearchDepth=extraSearchDepth,
                                         explorePopularSeeds=int(explorePopularSeeds),
                                         stopOnFirstHit=int(stopOnFirstHit))
        self._h = _check(lib().snapgpu_aligner_create(device, index._h, C.byref(self.params)), "aligner_create")

    def AlignReads(self, reads, out=None):
        """Batched AlignRead -> numpy structured array of RESULT_DTYPE (written into `out`
        when given: a caller streaming batches reuses one record buffer)."""
        n = reads.n
        if out is None:
            out = np.zeros(max(1, n), dtype=RESULT_DTYPE)
        elif out.dtype != RESULT_DTYPE or len(out) < n or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous RESULT_DTYPE array of at least reads.n records")
        if n:
            _check(lib().snapgpu_align_batch(self._h, reads._p, out.ctypes.data_as(C.POINTER(_ffi.Result))),
                   "align_batch")
        return out[:n]

    def submit(self, reads, out):
        """Queue a batch (snapgpu_align_batch_submit); `reads` and `out` stay owned by the caller
        and must not change until wait()."""
        if out.dtype != RESULT_DTYPE or len(out) < reads.n or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous RESULT_DTYPE array of at least reads.n records")
        if reads.n:
            _check(lib().snapgpu_align_batch_submit(self._h, reads._p, out.ctypes.data_as(C.POINTER(_ffi.Result))),
                   "align_batch_submit")

    def wait(self):
        """Finish every submitted batch (snapgpu_align_batch_wait)."""
        _check(lib().snapgpu_align_batch_wait(self._h), "align_batch_wait")

    def AlignReadsEx(self, reads, search=None, maxHitsToGet=0):
        """Batched form of the richer AlignRead (BaseAligner.h:73-86): per-read search
        windows (see search_array) and up to maxHitsToGet multi-hits per read.
        -> (results, multiHitsFound int32[n], multiHits MULTI_HIT_DTYPE[n, maxHitsToGet])."""
        n = reads.n
        out = np.zeros(max(1, n), dtype=RESULT_DTYPE)
        found = np.zeros(max(1, n), dtype=np.int32)
        hits = np.zeros((max(1, n), max(1, maxHitsToGet)), dtype=MULTI_HIT_DTYPE)
        srch = search_array(search, n)
        if n:
            _check(lib().snapgpu_align_batch_ex(self._h, reads._p, None if srch is None else srch.ctypes.data,
                                                maxHitsToGet, out.ctypes.data, found.ctypes.data,
                                                hits.ctypes.data), "align_batch_ex")
        return out[:n], found[:n], hits[:n, :maxHitsToGet]

    def AlignRead(self, bases, quals=None):
        """-> (AlignmentResult, genomeLocation, direction, score, mapq) for one read."""
        if quals is None:
            quals = "I" * len(bases)
        r = self.AlignReads(Reads.from_list([(bases, quals)]))[0]
        return int(r["result"]), int(r["location"]), int(r["direction"]), int(r["score"]), int(r["mapq"])

    def Cigars(self, reads, locations, directions, useM=False):
        """CIGARs as SAMFormat::computeCigarString computes them (SAM.cpp:1162-1230), on
        the GPU, for explicit (location, direction) per read (see cigar_inputs for the
        SAM writer's rules).  -> Cigars(editDistance int32[n], nOps uint32[n],
        ops uint32[n, 64] BAM ops)."""
        n = reads.n
        loc = np.ascontiguousarray(locations, dtype=np.uint32)
        dr = np.ascontiguousarray(directions, dtype=np.uint8)
        assert loc.shape == (n,) and dr.shape == (n,)
        c = Cigars.empty(n)
        if n:
            _check(lib().snapgpu_cigar_batch(self._h, reads._p, loc.ctypes.data, dr.ctypes.data, int(useM),
                                             c.editDistance.ctypes.data, c.nOps.ctypes.data, c.ops.ctypes.data),
                   "cigar_batch")
        return c

    def bucket_info(self):
        """The device bucket image of the seed tables (snapgpu_aligner_bucket_info) as a dict."""
        b = _ffi.BucketInfo()
        _check(lib().snapgpu_aligner_bucket_info(self._h, C.byref(b)), "bucket_info")
        return {f: getattr(b, f) for f, _ in b._fields_}

    def lookup_seeds(self, seeds, mode=0):
        """GenomeIndex::lookupSeed of ACGT seeds on the device, through the bucket image
        (snapgpu_aligner_lookup_seeds; mode 0 = lane per seed, 1 = wave per seed, 2 = four lanes per line).
        -> (uint64[n, 6] {nFwd, nRc, hashFwd, hashRc, firstFwd, firstRc}, uint32[n] lines)."""
        seeds = [s.encode() if isinstance(s, str) else bytes(s) for s in seeds]
        n = len(seeds)
        out = np.zeros((max(1, n), 6), dtype=np.uint64)
        lines = np.zeros(max(1, n), dtype=np.uint32)
        if n:
            _check(lib().snapgpu_aligner_lookup_seeds(self._h, b"".join(seeds), n, int(mode), out.ctypes.data,
                                                       lines.ctypes.data), "lookup_seeds")
        return out[:n], lines[:n]

    def gather_peak_ms(self, n_loads):
        """Diagnostic: best-of-3 time (ms) of n_loads independent random 64-byte bucket-line
        loads from the resident bucket image (roofline calibration for the seed lookups)."""
        ms = C.c_double()
        _check(lib().snapgpu_gather_peak(self._h, int(n_loads), C.byref(ms)), "gather_peak")
        return ms.value

    def set_overlap(self, overlap):
        """Let the pass sets of the two streams run concurrently (default) or one after the other."""
        _check(lib().snapgpu_aligner_set_overlap(self._h, int(bool(overlap))), "set_overlap")

    def debug_trip(self, read_index=0xffffffff):
        """Test hook: trip this aligner's device watchdog when read `read_index` of a batch starts."""
        _check(lib().snapgpu_aligner_debug_trip(self._h, int(read_index)), "debug_trip")

    def copy_peak_ms(self, nbytes):
        """Diagnostic: best-of-3 time (ms) of a streaming copy of nbytes (read nbytes + write nbytes)."""
        ms = C.c_double()
        _check(lib().snapgpu_copy_peak(self._h, int(nbytes), C.byref(ms)), "copy_peak")
        return ms.value

    def cigar_ms(self):
        ms = C.c_double()
        _check(lib().snapgpu_cigar_last_ms(self._h, C.byref(ms)), "cigar_last_ms")
        return ms.value

    # resident path (bench): upload once, time only the GPU passes
    def upload(self, reads):
        return DeviceReads(self, reads)

    def timing(self):
        t = _ffi.Timing()
        lib().snapgpu_last_timing(self._h, C.byref(t))
        return {f: getattr(t, f) for f, _ in t._fields_}

    PHASES = ("setup", "lookup", "insert", "score", "pop", "n_lv_forced_unknown_lowk", "stage", "lv_fwd", "lv_rev", "apply",
              "writeback", "out", "n_pass", "n_cand", "n_lv_forced_unknown_second", "n_pass16", "n_pass32", "n_pass64", "rows_fwd",
              "rows_rev", "n_score_calls", "n_forced", "n_popped", "n_succ", "passloop", "select", "fetch", "seedloop",
              "n_batch", "rank", "n_elems_forced", "candlist", "succ", "nearby", "prob", "fails", "n_fail_steps",
              "succ_tail", "n_pass_forced", "passloop_forced", "heavy_read_cycles", "n_heavy_reads", "n_cand_forced",
              "read_cycles", "n_filter", "n_lv_forced", "n_lv_forced_known", "n_filter_results")

    def phase_cycles(self, reset=True):
        """Diagnostic per-phase shader-cycle sums (needs SNAPGPU_PHASES=1 at construction)."""
        buf = (C.c_uint64 * 48)()
        _check(lib().snapgpu_phase_cycles(self._h, buf, 48, int(reset)), "phase_cycles")
        return {k: int(buf[i]) for i, k in enumerate(self.PHASES)}

    def stats(self):
        s = _ffi.AlignerStats()
        lib().snapgpu_aligner_get_stats(self._h, C.byref(s))
        return {f: getattr(s, f) for f, _ in s._fields_}

    # getters of SNAPLib/Aligner.h:62-77
    def getNHashTableLookups(self):
        return self.stats()["nHashTableLookups"]

    def getLocationsScored(self):
        return self.stats()["nLocationsScored"]

    def getNHitsIgnoredBecauseOfTooHighPopularity(self):
        return self.stats()["nHitsIgnoredBecauseOfTooHighPopularity"]

    def getNReadsIgnoredBecauseOfTooManyNs(self):
        return self.stats()["nReadsIgnoredBecauseOfTooManyNs"]

    def getNIndelsMerged(self):
        return self.stats()["nIndelsMerged"]

    def getMaxK(self):
        return lib().snapgpu_aligner_max_k(self._h)

    def getName(self):
        return lib().snapgpu_aligner_name(self._h).decode()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_aligner_free(self._h)
            self._h = None


def paired_params(**kw):
    """snapgpu_paired_params_t with the paired CLI defaults, overridden by kw."""
    p = _ffi.PairedParams()
    lib().snapgpu_paired_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class PairedAligner:
    """GPU ChimericPairedEndAligner over an IntersectingPairedEndAligner, constructed as
    PairedAligner.cpp:462-482 does (SNAPLib/ChimericPairedEndAligner.h, IntersectingPairedEndAligner.h).
    align() is ChimericPairedEndAligner::align for every pair; intersect() the intersecting aligner
    alone.  Keyword arguments: snapgpu_paired_params_t fields (maxHits, maxK, maxSeedsToUse,
    extraSearchDepth, minSpacing, maxSpacing, maxBigHits, maxCandidatePoolSize, maxReadSize,
    forceSpacing, seedCoverage)."""

    def __init__(self, index, device=0, **kw):
        self.index = index
        self.params = paired_params(**kw)
        self._h = _check(lib().snapgpu_paired_aligner_create(device, index._h, C.byref(self.params)),
                         "paired_aligner_create")

    def _run(self, fn, reads0, reads1, what):
        if reads0.n != reads1.n:
            raise ValueError("the two read batches differ in length")
        out = np.zeros(max(1, reads0.n), dtype=PAIR_RESULT_DTYPE)
        if reads0.n:
            _check(fn(self._h, reads0._p, reads1._p, out.ctypes.data), what)
        return out[:reads0.n]

    def align(self, reads0, reads1):
        return self._run(lib().snapgpu_paired_align_batch, reads0, reads1, "paired_align_batch")

    def intersect(self, reads0, reads1):
        return self._run(lib().snapgpu_paired_intersect_batch, reads0, reads1, "paired_intersect_batch")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_paired_aligner_free(self._h)
            self._h = None


SEED_RUN_DTYPE = np.dtype([("location", "<u4"), ("minOffset", "<u2"), ("maxOffset", "<u2"), ("count", "<u2"),
                           ("direction", "u1"), ("reserved", "u1")])


def charseeds_params(**kw):
    """snapgpu_charseeds_params_t: the partial aligner of PairedAligner.cpp:518-527 by default."""
    p = _ffi.CharSeedsParams()
    lib().snapgpu_charseeds_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def characterize_seeds(aligner, reads, read_list=None, **kw):
    """BaseAligner::CharacterizeSeeds (BaseAligner.cpp:206-508) on the GPU over `reads` (or the
    reads at indices read_list), on the index of `aligner`.  -> (start uint64[n+1],
    nForward uint32[n], flags uint32[n], runs SEED_RUN_DTYPE[...]): read i's map entries are
    runs[start[i]:start[i+1]], the first nForward[i] of them from `map`, the rest from `mapRC`."""
    p = charseeds_params(**kw)
    lst = None if read_list is None else np.ascontiguousarray(read_list, dtype=np.uint64)
    h = lib().snapgpu_characterize_seeds(aligner._h, reads._p, None if lst is None else lst.ctypes.data,
                                         0 if lst is None else len(lst), C.byref(p))
    if not h:
        raise SnapGpuError(f"characterize_seeds: {last_error()}")
    try:
        r = h.contents
        n = r.n
        start = np.ctypeslib.as_array(r.start, shape=(n + 1,)).copy()
        nfwd = np.ctypeslib.as_array(r.nForward, shape=(max(1, n),))[:n].copy()
        flags = np.ctypeslib.as_array(r.flags, shape=(max(1, n),))[:n].copy()
        runs = np.zeros(r.nRuns, dtype=SEED_RUN_DTYPE)
        if r.nRuns:
            C.memmove(runs.ctypes.data, r.runs, r.nRuns * SEED_RUN_DTYPE.itemsize)
    finally:
        lib().snapgpu_seed_runs_free(h)
    return start, nfwd, flags, runs


class DeviceReads:
    def __init__(self, aligner, reads):
        self.aligner = aligner
        self.n = reads.n
        self._h = _check(lib().snapgpu_reads_upload(aligner._h, reads._p), "reads_upload")

    def run(self):
        """Launch the GPU passes (asynchronous)."""
        _check(lib().snapgpu_align_resident(self.aligner._h, self._h), "align_resident")

    def synchronize(self):
        _check(lib().snapgpu_synchronize(self.aligner._h), "synchronize")

    def results(self):
        out = np.zeros(max(1, self.n), dtype=RESULT_DTYPE)
        _check(lib().snapgpu_results_download(self.aligner._h, self._h,
                                              out.ctypes.data_as(C.POINTER(_ffi.Result))), "results_download")
        return out[:self.n]

    def run_cigars(self, useM=False):
        """CIGARs of the records the last run() left in HBM (asynchronous)."""
        _check(lib().snapgpu_cigar_resident(self.aligner._h, self._h, int(useM)), "cigar_resident")

    def cigars(self):
        c = Cigars.empty(self.n)
        _check(lib().snapgpu_cigar_download(self.aligner._h, self._h, c.editDistance.ctypes.data,
                                            c.nOps.ctypes.data, c.ops.ctypes.data), "cigar_download")
        return c

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_device_reads_free(self._h)
            self._h = None


CIGAR_OPS = "MIDNSHP=X"   # BAM op codes (SAM spec; BAMAlignment::CigarToCode)


class Cigars:
    """Per-read CIGAR results: editDistance (NM, -1 = "*"), nOps, ops (BAM-encoded)."""

    def __init__(self, editDistance, nOps, ops):
        self.editDistance, self.nOps, self.ops = editDistance, nOps, ops

    @classmethod
    def empty(cls, n):
        return cls(np.full(max(1, n), -1, dtype=np.int32)[:n], np.zeros(max(1, n), dtype=np.uint32)[:n],
                   np.zeros((max(1, n), _ffi.CIGAR_MAX_OPS), dtype=np.uint32)[:n])

    def string(self, i):
        """COMPACT_CIGAR_STRING form (LandauVishkin.cpp:49-62), or "*"."""
        if self.editDistance[i] < 0:
            return "*"
        return "".join(f"{int(o) >> 4}{CIGAR_OPS[int(o) & 15]}" for o in self.ops[i, :self.nOps[i]])


def cigar_inputs(results):
    """(locations, directions) the SAM writer computes CIGARs for (SAM.cpp:1007-1048,
    855-883): writeRead's own location, the forward read unless the read is mapped RC."""
    loc = np.ascontiguousarray(results["location"], dtype=np.uint32)
    mapped = (results["result"] != NotFound) & (loc != 0xFFFFFFFF)
    return loc, np.where(mapped, results["direction"], 0).astype(np.uint8)


def sam_header(index, command_line, version, sorted_output=False, rg_line=None):
    """SAM header (SAMFormat::writeHeader, SAM.cpp:700-800) for a FASTQ input -> bytes."""
    used = C.c_uint64()
    args = [index._h, int(sorted_output), command_line.encode(), version.encode(),
            None if rg_line is None else rg_line.encode()]
    lib().snapgpu_sam_header(*args, None, 0, C.byref(used))
    buf = C.create_string_buffer(max(1, used.value))
    _check(lib().snapgpu_sam_header(*args, buf, used.value, C.byref(used)), "sam_header")
    return C.string_at(buf, used.value)


def sam_format(index, reads, ids, results, cigars, read_group="FASTQ", clip=None, timing=None):
    """SAM lines (SAMFormat::writeRead, SAM.cpp:1007-1155) of single-end genome
    alignments -> bytes.  ids: list of read ids (str/bytes); clip: the (frontClipped,
    unclippedLength) pair Reads.clip returned, or None for unclipped reads; timing: a dict that
    receives the seconds spent in the C formatter ("format_s")."""
    n = reads.n
    idb = [i.encode() if isinstance(i, str) else bytes(i) for i in ids]
    assert len(idb) == n
    lens = np.array([len(x) for x in idb], dtype=np.uint32)
    offs = np.zeros(max(1, n), dtype=np.uint64)
    if n > 1:
        offs[1:n] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = b"".join(idb) + b"\0"
    res = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    used = C.c_uint64()
    rg = None if read_group is None else read_group.encode()
    args = [index._h, reads._p, blob, offs.ctypes.data, lens.ctypes.data, res.ctypes.data,
            cigars.editDistance.ctypes.data, cigars.nOps.ctypes.data, cigars.ops.ctypes.data, rg]
    fn = lib().snapgpu_sam_format
    if clip is not None:
        front = np.ascontiguousarray(clip[0], dtype=np.uint32)
        full = np.ascontiguousarray(clip[1], dtype=np.uint32)
        assert front.shape == (n,) and full.shape == (n,)
        args += [front.ctypes.data, full.ctypes.data]
        fn = lib().snapgpu_sam_format_clipped
    # one formatting pass with a generous (uninitialised) buffer; a second only if it was too small
    cap = int(lens.sum()) + 2 * int(reads._p.contents.totalBytes) + n * 512
    buf = np.empty(max(1, cap), dtype=np.uint8)
    t0 = time.perf_counter()
    rc = fn(*args, buf.ctypes.data, cap, C.byref(used))
    if rc != 0:
        buf = np.empty(max(1, used.value), dtype=np.uint8)
        t0 = time.perf_counter()
        _check(fn(*args, buf.ctypes.data, used.value, C.byref(used)), "sam_format")
    if timing is not None:
        timing["format_s"] = time.perf_counter() - t0
    return buf[:used.value].tobytes()


def lv_batch(direction, tasks, device=0, engine="byte"):
    """LandauVishkin<direction>::computeEditDistance on the GPU.

    tasks: list of (text, pattern, quals, k) (str/bytes).  -> list of (score, netIndel, prob).
    engine "byte": the byte-compare LV of align_kernel<512>; "bitplane": the production LV of
    align_kernel<128> (patterns of 1..127 bases)."""
    n = len(tasks)
    texts, pats, quals = bytearray(), bytearray(), bytearray()
    toff, tlen, poff, plen, ks = [], [], [], [], []
    for t, p, q, k in tasks:
        t = t.encode() if isinstance(t, str) else bytes(t)
        p = p.encode() if isinstance(p, str) else bytes(p)
        q = q.encode() if isinstance(q, str) else bytes(q)
        toff.append(len(texts)); tlen.append(len(t)); texts += t
        poff.append(len(pats)); plen.append(len(p)); pats += p; quals += q[:len(p)].ljust(len(p), b"!")
        ks.append(k)
    texts += b"\0" * 16; pats += b"\0" * 16; quals += b"\0" * 16
    A64, A32, AI = C.c_uint64 * n, C.c_uint32 * n, C.c_int32 * n
    os_, on, op = AI(), AI(), (C.c_double * n)()
    fn = lib().snapgpu_lv_batch if engine == "byte" else lib().snapgpu_lv_group_batch
    _check(fn(device, direction, n, bytes(texts), A64(*toff), A32(*tlen), bytes(pats),
              bytes(quals), A64(*poff), A32(*plen), AI(*ks), os_, on, op), "lv_batch")
    return [(os_[i], on[i], op[i]) for i in range(n)]


def compute_mapq(pAll, pBest, score, popularSeedsSkipped):
    return lib().snapgpu_compute_mapq(pAll, pBest, score, popularSeedsSkipped)


class Gtf:
    """Genome annotation (SNAPLib/GTFReader: exon lines -> transcripts with introns)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load(cls, path):
        return cls(_check(lib().snapgpu_gtf_load(str(path).encode()), "gtf_load"))

    def counts(self):
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(lib().snapgpu_gtf_counts(self._h, C.byref(a), C.byref(b), C.byref(c)), "gtf_counts")
        return {"features": a.value, "transcripts": b.value, "genes": c.value}

    def write_transcriptome(self, genome, path):
        """GTFReader::BuildTranscriptome: the transcriptome FASTA `snap-rna transcriptome` indexes.
        genome: a Genome or a raw genome handle (GenomeIndex.genome_handle())."""
        g = genome._h if isinstance(genome, Genome) else genome
        _check(lib().snapgpu_gtf_write_transcriptome(self._h, g, str(path).encode()), "gtf_write_transcriptome")

    def genomic_position(self, transcript_id, pos, span):
        out = C.c_uint32()
        _check(lib().snapgpu_gtf_genomic_position(self._h, transcript_id.encode(), pos, span, C.byref(out)),
               "gtf_genomic_position")
        return out.value

    def splice_cigar(self, transcript_id, pos, tokens):
        """insertSpliceJunctions over [(count, op), ...] -> CIGAR string."""
        counts = (C.c_uint32 * max(1, len(tokens)))(*[int(c) for c, _ in tokens])
        ops = "".join(o for _, o in tokens).encode()
        used = C.c_uint64()
        buf = C.create_string_buffer(4096)
        _check(lib().snapgpu_gtf_splice_cigar(self._h, transcript_id.encode(), pos, len(tokens), counts, ops, buf,
                                              4096, C.byref(used)), "gtf_splice_cigar")
        return buf.value.decode()

    def write_counts(self, prefix):
        """GTFReader::WriteReadCounts: <prefix>.{transcript,gene,junction}_{id,name}.counts.txt."""
        _check(lib().snapgpu_gtf_write_counts(self._h, str(prefix).encode()), "gtf_write_counts")

    def reset_counts(self):
        _check(lib().snapgpu_gtf_reset_counts(self._h), "gtf_reset_counts")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_gtf_free(self._h)
            self._h = None


def sam_sort_records(index, text):
    """`-so`: SAM record lines (bytes, no header) stable-sorted by SAMFormat::getSortInfo's location."""
    used = C.c_uint64()
    buf = C.create_string_buffer(max(1, len(text)))
    _check(lib().snapgpu_sam_sort_records(index._h, text, len(text), buf, len(text), C.byref(used)), "sam_sort_records")
    return C.string_at(buf, used.value)


class Contaminants:
    """The contamination database's counts (`-ct`, ContaminationFilter): contaminant alignments per
    contig of the contamination index, accumulated over the product-path calls given
    contamination=(aligner, this); write() leaves `<prefix>.contaminants.txt` as the reference."""

    def __init__(self, contamination_index):
        self._index = contamination_index
        self._h = _check(lib().snapgpu_contaminants_create(contamination_index._h), "contaminants_create")

    def add(self, location):
        """ContaminationFilter::AddAlignment of one aligned location of the contamination genome."""
        _check(lib().snapgpu_contaminants_add(self._h, int(location)), "contaminants_add")

    def text(self):
        used = C.c_uint64()
        _check(lib().snapgpu_contaminants_format(self._h, None, 0, C.byref(used)), "contaminants_format")
        buf = C.create_string_buffer(max(1, used.value))
        _check(lib().snapgpu_contaminants_format(self._h, buf, used.value, C.byref(used)), "contaminants_format")
        return C.string_at(buf, used.value).decode()

    def write(self, output_template):
        _check(lib().snapgpu_contaminants_write(self._h, None if output_template is None else str(output_template).encode()),
               "contaminants_write")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().snapgpu_contaminants_free(self._h)
            self._h = None


def _contamination_opts(o, contamination):
    if contamination is not None:
        aligner, counts = contamination
        o.contaminationAligner = aligner._h
        o.contaminants = counts._h


def single_options(**kw):
    o = _ffi.SingleOptions()
    lib().snapgpu_single_options_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v.encode() if isinstance(v, str) else v)
    return o


def single_align(genome_aligner, transcriptome_aligner, gtf, reads, sam_path, contamination=None, **options):
    """`snap-rna single` (SingleAligner.cpp:141-320) over a FASTQ batch, both AlignRead calls and
    the CIGARs on the GPU; writes sam_path.  options: SingleOptions fields; contamination:
    (BaseAligner over the contamination index, Contaminants) for `-ct`.  -> stats dict."""
    o = single_options(**options)
    _contamination_opts(o, contamination)
    st = _ffi.SingleStats()
    _check(lib().snapgpu_single_align(genome_aligner._h, transcriptome_aligner._h, gtf._h, reads._p, C.byref(o),
                                      str(sam_path).encode(), C.byref(st)), "single_align")
    return {f: getattr(st, f) for f, _ in st._fields_}


RNA_PAIR_RESULT_DTYPE = np.dtype([
    ("location", "<u4", (2,)), ("tlocation", "<u4", (2,)), ("score", "<i4", (2,)), ("mapq", "<i4", (2,)),
    ("status", "u1", (2,)), ("direction", "u1", (2,)), ("isTranscriptome", "u1", (2,)), ("fromAlignTogether", "u1"),
    ("alignedAsPair", "u1"), ("useful", "u1"), ("reserved", "u1", (7,)),
])
assert RNA_PAIR_RESULT_DTYPE.itemsize == 48


def rna_paired_options(**kw):
    o = _ffi.RnaPairedOptions()
    lib().snapgpu_rna_paired_options_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v.encode() if isinstance(v, str) else v)
    return o


def rna_paired_align(paired_aligner, transcriptome_aligner, gtf, reads0, reads1, sam_path=None, contamination=None,
                     **options):
    """`snap-rna paired` (PairedAligner.cpp:405-689) over a FASTQ pair batch: the transcriptome and
    genome aligners, the seed census of FindPartialMatches and the CIGARs on the GPU; writes
    sam_path (if given) and advances gtf's read counters.  -> (RNA_PAIR_RESULT_DTYPE[n], stats)."""
    o = rna_paired_options(**options)
    _contamination_opts(o, contamination)   # (PairedAligner over the contamination index, Contaminants): -ct
    st = _ffi.RnaPairedStats()
    out = np.zeros(max(1, reads0.n), dtype=RNA_PAIR_RESULT_DTYPE)
    _check(lib().snapgpu_rna_paired_align(paired_aligner._h, transcriptome_aligner._h, gtf._h, reads0._p, reads1._p,
                                          C.byref(o), None if sam_path is None else str(sam_path).encode(),
                                          out.ctypes.data, C.byref(st)), "rna_paired_align")
    return out[:reads0.n], {f: getattr(st, f) for f, _ in st._fields_}

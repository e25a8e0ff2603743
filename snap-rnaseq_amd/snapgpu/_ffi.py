"""ctypes declarations of the C ABI in include/snapgpu.h.

The product library is ``libsnapgpu.so`` built in-tree next to this file by
``snap-rnaseq_amd/Makefile`` (hipcc for gfx950 + g++ for the host side).  There is
no Python or CPU fallback for the aligner: if the library (or a GPU) is missing,
creating an aligner raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SNAPGPU_LIB", os.path.join(_HERE, "libsnapgpu.so"))


class Result(C.Structure):
    """snapgpu_result_t -- one BaseAligner::AlignRead outcome (BaseAligner.cpp:510-938)."""
    _fields_ = [
        ("location", C.c_uint32),
        ("score", C.c_int32),
        ("mapq", C.c_int32),
        ("result", C.c_uint8),
        ("direction", C.c_uint8),
        ("flags", C.c_uint8),
        ("reserved", C.c_uint8),
        ("nLookups", C.c_uint32),
        ("nLocationsScored", C.c_uint32),
        ("popularSeedsSkipped", C.c_uint16),
        ("nHitsIgnored", C.c_uint16),
        ("nProbes", C.c_uint32),
        ("nHitWords", C.c_uint32),
        ("nOverflowLists", C.c_uint32),
        ("nElements", C.c_uint32),
        ("reserved2", C.c_uint32),
        ("probabilityOfAllCandidates", C.c_double),
        ("probabilityOfBestCandidate", C.c_double),
    ]


class AlignerParams(C.Structure):
    _fields_ = [
        ("maxHitsToConsider", C.c_uint32),
        ("maxK", C.c_uint32),
        ("maxReadSize", C.c_uint32),
        ("maxSeedsToUse", C.c_uint32),
        ("maxSeedCoverage", C.c_double),
        ("extraSearchDepth", C.c_uint32),
        ("explorePopularSeeds", C.c_uint32),
        ("stopOnFirstHit", C.c_uint32),
    ]


class PairedParams(C.Structure):
    """snapgpu_paired_params_t (PairedAligner.cpp:462-482 construction arguments)."""
    _fields_ = [
        ("maxHits", C.c_uint32), ("maxK", C.c_uint32), ("maxSeedsToUse", C.c_uint32),
        ("extraSearchDepth", C.c_uint32), ("minSpacing", C.c_uint32), ("maxSpacing", C.c_uint32),
        ("maxBigHits", C.c_uint32), ("maxCandidatePoolSize", C.c_uint32), ("maxReadSize", C.c_uint32),
        ("forceSpacing", C.c_uint32), ("seedCoverage", C.c_double),
    ]


class SynthGenomeParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("totalBases", C.c_uint64),
        ("nContigs", C.c_uint32),
        ("nRepeatFamilies", C.c_uint32),
        ("repeatFraction", C.c_double),
        ("maxDivergence", C.c_double),
        ("nRunFraction", C.c_double),
        ("chromosomePadding", C.c_uint32),
    ]


class SynthReadsParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("nReads", C.c_uint64),
        ("readLength", C.c_uint32),
        ("qualityChar", C.c_uint32),
        ("baseErrorRate", C.c_double),
        ("mutationRate", C.c_double),
        ("indelFraction", C.c_double),
        ("indelExtend", C.c_double),
        ("randomReadFraction", C.c_double),
    ]


class Reads(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("totalBytes", C.c_uint64),
        ("bases", C.c_void_p),
        ("quals", C.c_void_p),
        ("offsets", C.POINTER(C.c_uint64)),
        ("lengths", C.POINTER(C.c_uint32)),
        ("truthLocation", C.POINTER(C.c_uint32)),
        ("truthDirection", C.POINTER(C.c_uint8)),
        ("frontClipped", C.POINTER(C.c_uint32)),
        ("unclippedLength", C.POINTER(C.c_uint32)),
        ("clipping", C.c_int32),
        ("nUploads", C.c_uint32),
        ("ids", C.c_void_p),
        ("idOffsets", C.POINTER(C.c_uint64)),
        ("idLengths", C.POINTER(C.c_uint32)),
        ("hostFlags", C.c_uint32),
        ("reserved_", C.c_uint32),
    ]


class IndexInfo(C.Structure):
    _fields_ = [
        ("nBases", C.c_uint32),
        ("seedLen", C.c_uint32),
        ("nHashTables", C.c_uint32),
        ("chromosomePadding", C.c_uint32),
        ("overflowTableSize", C.c_uint64),
        ("totalHashSlots", C.c_uint64),
        ("totalUsedSlots", C.c_uint64),
        ("nPieces", C.c_int32),
        ("hasIupac", C.c_uint32),
    ]


class IndexView(C.Structure):
    _fields_ = [
        ("slots", C.c_void_p),
        ("tableBase", C.c_void_p),
        ("tableSize", C.c_void_p),
        ("overflow", C.c_void_p),
        ("genome", C.c_void_p),
        ("pieceOffsets", C.c_void_p),
        ("nBases", C.c_uint32),
        ("seedLen", C.c_uint32),
        ("nHashTables", C.c_uint32),
        ("chromosomePadding", C.c_uint32),
        ("nPieces", C.c_int32),
        ("pad_", C.c_uint32),
        ("overflowTableSize", C.c_uint64),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("mainKernelMs", C.c_double),
        ("spillKernelMs", C.c_double),
        ("fixupMs", C.c_double),
        ("nSpilled", C.c_uint64),
        ("nMapqFixed", C.c_uint64),
        ("lookupKernelMs", C.c_double),
        ("lookupSeeds", C.c_uint64),
        ("lookupProbes", C.c_uint64),
        ("lookupOverflowReads", C.c_uint64),
        ("nLaunches", C.c_uint64),
        ("wallMs", C.c_double),
        ("mainKernelBusyMs", C.c_double),
        ("lookupKernelBusyMs", C.c_double),
        ("nByteReads", C.c_uint64),
        ("nArenaOverflow", C.c_uint64),
        ("nNulReads", C.c_uint64),
        ("nUnwritten", C.c_uint64),
    ]


class SingleOptions(C.Structure):
    _fields_ = [
        ("clipping", C.c_int32),
        ("confDiff", C.c_uint32),
        ("maxDist", C.c_uint32),
        ("minPercentAbovePhred", C.c_float),
        ("minPhred", C.c_uint32),
        ("phredOffset", C.c_uint32),
        ("useM", C.c_uint32),
        ("sortOutput", C.c_uint32),
        ("readGroup", C.c_char_p),
        ("commandLine", C.c_char_p),
        ("version", C.c_char_p),
        ("contaminationAligner", C.c_void_p),
        ("contaminants", C.c_void_p),
    ]


class RnaPairedOptions(C.Structure):
    _fields_ = [
        ("clipping", C.c_int32), ("confDiff", C.c_uint32), ("maxDist", C.c_uint32), ("minSpacing", C.c_uint32),
        ("maxSpacing", C.c_uint32), ("forceSpacing", C.c_uint32), ("minPercentAbovePhred", C.c_float),
        ("minPhred", C.c_uint32), ("phredOffset", C.c_uint32), ("useM", C.c_uint32), ("maxHitsToGet", C.c_uint32),
        ("ignoreMismatchedIDs", C.c_uint32), ("readGroup", C.c_char_p), ("commandLine", C.c_char_p),
        ("version", C.c_char_p), ("contaminationAligner", C.c_void_p), ("contaminants", C.c_void_p),
        ("sortOutput", C.c_uint32),
    ]


class RnaPairedStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("totalPairs", "usefulPairs", "singleHits", "multiHits", "notFound",
                                          "transcriptomeRecords", "partialPairs", "partialMatches", "seedRuns")] + \
               [(f, C.c_double) for f in ("alignMs", "filterMs", "seedMs", "cigarMs", "writeMs", "wallMs", "prepMs",
                                           "countMs")] + [("subBatches", C.c_uint64)] + \
               [(f, C.c_double) for f in ("cigarGpuMs", "spliceMs")] + [("countedPairs", C.c_uint64)]


class SingleStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("totalReads", "usefulReads", "singleHits", "multiHits", "notFound",
                                          "transcriptomeRecords")] + \
               [(f, C.c_double) for f in ("alignMs", "cigarMs", "filterMs", "writeMs", "wallMs", "prepMs", "formatMs", "ioMs")]


class SeedRuns(C.Structure):
    """snapgpu_seed_runs_t (BaseAligner::CharacterizeSeeds maps as run records)."""
    _fields_ = [("n", C.c_uint64), ("start", C.POINTER(C.c_uint64)), ("nForward", C.POINTER(C.c_uint32)),
                ("flags", C.POINTER(C.c_uint32)), ("runs", C.c_void_p), ("nRuns", C.c_uint64)]


class CharSeedsParams(C.Structure):
    _fields_ = [("maxHits", C.c_uint32), ("maxK", C.c_uint32), ("numSeeds", C.c_uint32), ("maxReadSize", C.c_uint32),
                ("explorePopularSeeds", C.c_uint32), ("reserved", C.c_uint32)]


class AlignerStats(C.Structure):
    _fields_ = [
        ("nHashTableLookups", C.c_int64),
        ("nLocationsScored", C.c_int64),
        ("nHitsIgnoredBecauseOfTooHighPopularity", C.c_int64),
        ("nReadsIgnoredBecauseOfTooManyNs", C.c_int64),
        ("nIndelsMerged", C.c_int64),
        ("nReads", C.c_int64),
    ]


assert C.sizeof(Result) == 64, C.sizeof(Result)

class BucketInfo(C.Structure):   # snapgpu_bucket_info_t
    _fields_ = [("nSlots", C.c_uint64), ("nKeys", C.c_uint64), ("nBuckets", C.c_uint64),
                ("nOverflowBuckets", C.c_uint64), ("maxDisplacement", C.c_uint64), ("bytes", C.c_uint64),
                ("buildMs", C.c_double)]


# (name, restype, argtypes)
_PROTOS = [
    ("snapgpu_abi_version", C.c_int, []),
    ("snapgpu_last_error", C.c_char_p, []),
    ("snapgpu_host_threads", C.c_int, []),
    ("snapgpu_aligner_params_default", None, [C.POINTER(AlignerParams)]),
    ("snapgpu_genome_from_fasta", C.c_void_p, [C.c_char_p, C.c_uint32]),
    ("snapgpu_genome_synthetic", C.c_void_p, [C.POINTER(SynthGenomeParams)]),
    ("snapgpu_genome_write_fasta", C.c_int, [C.c_void_p, C.c_char_p]),
    ("snapgpu_genome_free", None, [C.c_void_p]),
    ("snapgpu_genome_nbases", C.c_uint32, [C.c_void_p]),
    ("snapgpu_genome_bases", C.c_void_p, [C.c_void_p]),
    ("snapgpu_genome_npieces", C.c_int, [C.c_void_p]),
    ("snapgpu_genome_piece_offset", C.c_uint32, [C.c_void_p, C.c_int]),
    ("snapgpu_genome_piece_name", C.c_char_p, [C.c_void_p, C.c_int]),
    ("snapgpu_index_build", C.c_void_p, [C.c_void_p, C.c_int, C.c_int]),
    ("snapgpu_index_build_ex", C.c_void_p, [C.c_void_p, C.c_int, C.c_int, C.c_double]),
    ("snapgpu_index_load", C.c_void_p, [C.c_char_p]),
    ("snapgpu_index_share", C.c_int, [C.c_void_p, C.c_char_p]),
    ("snapgpu_index_attach", C.c_void_p, [C.c_char_p]),
    ("snapgpu_index_genome", C.c_void_p, [C.c_void_p]),
    ("snapgpu_index_save", C.c_int, [C.c_void_p, C.c_char_p]),
    ("snapgpu_index_free", None, [C.c_void_p]),
    ("snapgpu_index_get_info", C.c_int, [C.c_void_p, C.POINTER(IndexInfo)]),
    ("snapgpu_index_get_view", C.c_int, [C.c_void_p, C.POINTER(IndexView)]),
    ("snapgpu_index_lookup", C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32]),
    ("snapgpu_reads_synthetic", C.POINTER(Reads), [C.c_void_p, C.POINTER(SynthReadsParams)]),
    ("snapgpu_reads_synthetic_pairs", C.c_int, [C.c_void_p, C.POINTER(SynthReadsParams), C.c_uint32, C.c_uint32,
                                                C.POINTER(C.POINTER(Reads)), C.POINTER(C.POINTER(Reads))]),
    ("snapgpu_reads_from_fastq", C.POINTER(Reads), [C.c_char_p]),
    ("snapgpu_reads_from_arrays", C.POINTER(Reads), [C.c_uint64, C.c_char_p, C.c_char_p,
                                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    ("snapgpu_reads_write_fastq", C.c_int, [C.POINTER(Reads), C.c_char_p]),
    ("snapgpu_reads_free", None, [C.POINTER(Reads)]),
    ("snapgpu_device_count", C.c_int, []),
    ("snapgpu_device_cu_count", C.c_int, [C.c_int]),
    ("snapgpu_aligner_create", C.c_void_p, [C.c_int, C.c_void_p, C.POINTER(AlignerParams)]),
    ("snapgpu_aligner_free", None, [C.c_void_p]),
    ("snapgpu_align_batch", C.c_int, [C.c_void_p, C.POINTER(Reads), C.POINTER(Result)]),
    ("snapgpu_align_batch_submit", C.c_int, [C.c_void_p, C.POINTER(Reads), C.POINTER(Result)]),
    ("snapgpu_align_batch_wait", C.c_int, [C.c_void_p]),
    ("snapgpu_align_batch_ex", C.c_int, [C.c_void_p, C.POINTER(Reads), C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.c_void_p]),
    ("snapgpu_reads_upload", C.c_void_p, [C.c_void_p, C.POINTER(Reads)]),
    ("snapgpu_device_reads_free", None, [C.c_void_p]),
    ("snapgpu_align_resident", C.c_int, [C.c_void_p, C.c_void_p]),
    ("snapgpu_results_download", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(Result)]),
    ("snapgpu_synchronize", C.c_int, [C.c_void_p]),
    ("snapgpu_last_timing", C.c_int, [C.c_void_p, C.POINTER(Timing)]),
    ("snapgpu_aligner_get_stats", C.c_int, [C.c_void_p, C.POINTER(AlignerStats)]),
    ("snapgpu_aligner_max_k", C.c_int, [C.c_void_p]),
    ("snapgpu_aligner_set_overlap", C.c_int, [C.c_void_p, C.c_int]),
    ("snapgpu_aligner_debug_trip", C.c_int, [C.c_void_p, C.c_uint32]),
    ("snapgpu_source_sha256", C.c_char_p, []),
    ("snapgpu_phase_cycles", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32, C.c_int]),
    ("snapgpu_aligner_name", C.c_char_p, [C.c_void_p]),
    ("snapgpu_lv_batch", C.c_int, [C.c_int, C.c_int, C.c_uint32, C.c_char_p, C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint32), C.c_char_p, C.c_char_p, C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
    ("snapgpu_lv_group_batch", C.c_int, [C.c_int, C.c_int, C.c_uint32, C.c_char_p, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint32), C.c_char_p, C.c_char_p, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
    ("snapgpu_compute_mapq", C.c_int, [C.c_double, C.c_double, C.c_int, C.c_int]),
    ("snapgpu_cigar_batch", C.c_int, [C.c_void_p, C.POINTER(Reads), C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                      C.c_void_p, C.c_void_p]),
    ("snapgpu_cigar_resident", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ("snapgpu_cigar_download", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("snapgpu_cigar_last_ms", C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    ("snapgpu_reads_clip", C.c_int, [C.POINTER(Reads), C.c_int, C.c_void_p, C.c_void_p]),
    ("snapgpu_sam_format_clipped", C.c_int, [C.c_void_p, C.POINTER(Reads), C.c_char_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("snapgpu_sam_header", C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_void_p,
                                     C.c_uint64, C.POINTER(C.c_uint64)]),
    ("snapgpu_gather_peak", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_double)]),
    ("snapgpu_aligner_bucket_info", C.c_int, [C.c_void_p, C.POINTER(BucketInfo)]),
    ("snapgpu_aligner_lookup_seeds", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p]),
    ("snapgpu_copy_peak", C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_double)]),
    ("snapgpu_selftest_timeout_path", C.c_int, []),
    ("snapgpu_sam_format", C.c_int, [C.c_void_p, C.POINTER(Reads), C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint64,
                                     C.POINTER(C.c_uint64)]),
]

_PROTOS += [
    ("snapgpu_gtf_load", C.c_void_p, [C.c_char_p]),
    ("snapgpu_gtf_free", None, [C.c_void_p]),
    ("snapgpu_gtf_counts", C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("snapgpu_gtf_write_transcriptome", C.c_int, [C.c_void_p, C.c_void_p, C.c_char_p]),
    ("snapgpu_gtf_genomic_position", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32,
                                               C.POINTER(C.c_uint32)]),
    ("snapgpu_gtf_splice_cigar", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_char_p,
                                           C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("snapgpu_single_options_default", None, [C.POINTER(SingleOptions)]),
    ("snapgpu_single_align", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(Reads), C.POINTER(SingleOptions),
                                       C.c_char_p, C.POINTER(SingleStats)]),
    ("snapgpu_aligner_index", C.c_void_p, [C.c_void_p]),
    ("snapgpu_aligner_get_params", C.c_int, [C.c_void_p, C.POINTER(AlignerParams)]),
    ("snapgpu_paired_params_default", None, [C.POINTER(PairedParams)]),
    ("snapgpu_paired_aligner_create", C.c_void_p, [C.c_int, C.c_void_p, C.POINTER(PairedParams)]),
    ("snapgpu_paired_aligner_free", None, [C.c_void_p]),
    ("snapgpu_paired_align_batch", C.c_int, [C.c_void_p, C.POINTER(Reads), C.POINTER(Reads), C.c_void_p]),
    ("snapgpu_paired_intersect_batch", C.c_int, [C.c_void_p, C.POINTER(Reads), C.POINTER(Reads), C.c_void_p]),
    ("snapgpu_paired_aligner_single", C.c_void_p, [C.c_void_p]),
    ("snapgpu_charseeds_params_default", None, [C.POINTER(CharSeedsParams)]),
    ("snapgpu_rna_paired_options_default", None, [C.POINTER(RnaPairedOptions)]),
    ("snapgpu_rna_paired_align", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(Reads), C.POINTER(Reads),
                                           C.POINTER(RnaPairedOptions), C.c_char_p, C.c_void_p,
                                           C.POINTER(RnaPairedStats)]),
    ("snapgpu_gtf_write_counts", C.c_int, [C.c_void_p, C.c_char_p]),
    ("snapgpu_sam_sort_records", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64,
                                           C.POINTER(C.c_uint64)]),
    ("snapgpu_contaminants_create", C.c_void_p, [C.c_void_p]),
    ("snapgpu_contaminants_free", None, [C.c_void_p]),
    ("snapgpu_contaminants_add", C.c_int, [C.c_void_p, C.c_uint32]),
    ("snapgpu_contaminants_write", C.c_int, [C.c_void_p, C.c_char_p]),
    ("snapgpu_contaminants_format", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("snapgpu_gtf_reset_counts", C.c_int, [C.c_void_p]),
    ("snapgpu_characterize_seeds", C.POINTER(SeedRuns), [C.c_void_p, C.POINTER(Reads), C.c_void_p, C.c_uint64,
                                                         C.POINTER(CharSeedsParams)]),
    ("snapgpu_seed_runs_free", None, [C.POINTER(SeedRuns)]),
]

CIGAR_MAX_OPS = 64   # SNAPGPU_CIGAR_MAX_OPS

EXPORTED_SYMBOLS = [p[0] for p in _PROTOS]

_lib = None


def lib():
    """Load libsnapgpu.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `make -C snap-rnaseq_amd` or __graft_entry__.build()")
        l = C.CDLL(LIB_PATH)
        for name, res, args in _PROTOS:
            if not hasattr(l, name):
                continue   # tests/test_capi.py asserts every symbol is exported
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        check_source_identity(l)
        _lib = l
    return _lib


class StaleLibraryError(OSError):
    pass


def check_source_identity(l):
    """The library embeds the identity of the sources it was built from (_srcsha.py); refuse it
    when the sources beside it differ (a stale prebuilt .so must not run in their place).
    SNAPGPU_ALLOW_STALE=1 turns the refusal into a warning (diagnostic builds only)."""
    from . import _srcsha
    want = _srcsha.source_sha256()
    if want is None or os.path.abspath(LIB_PATH) != os.path.join(_HERE, "libsnapgpu.so"):
        return   # no sources here, or an explicitly chosen variant build (SNAPGPU_LIB, tools/build_variant.sh)
    got = l.snapgpu_source_sha256().decode() if hasattr(l, "snapgpu_source_sha256") else None
    if got != want:
        msg = (f"{LIB_PATH} was built from other sources (embedded {str(got)[:16]}, sources here "
               f"{want[:16]}): rebuild with `make -C snap-rnaseq_amd`")
        if os.environ.get("SNAPGPU_ALLOW_STALE") == "1":
            import warnings
            warnings.warn(msg)
        else:
            raise StaleLibraryError(msg)


def last_error():
    return lib().snapgpu_last_error().decode(errors="replace")

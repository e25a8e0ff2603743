/*
 * snapgpu.h -- C ABI of the MI355X-native SNAP seed-and-extend hot path.
 *
 * This is the drop-in boundary for SNAPLib's `Aligner` / `BaseAligner` surface
 * (reference: SNAPLib/Aligner.h:54-80, SNAPLib/BaseAligner.h:44-142).  Every entry
 * point is plain C (pointers + sizes, no C++ or torch types) so that the
 * reference's C++ (apps/snap, SingleAlignerContext via AlignerExtension,
 * SNAPLib/AlignerContext.h:132-163) -- or ctypes / any FFI -- can bind it.
 * INTEGRATION.md shows the adapter a SNAPLib maintainer would add.
 *
 * Conventions
 *  - Functions returning int return SNAPGPU_OK (0) on success, a negative
 *    SNAPGPU_E* code on failure; snapgpu_last_error() gives the message.  The
 *    reference calls soft_exit() (SNAPLib/exit.cpp:27-31) where this API returns
 *    an error code instead (e.g. a read longer than maxReadSize,
 *    BaseAligner.cpp:609-613 -> per-read flag SNAPGPU_FLAG_READ_TOO_LONG).
 *  - Handles are opaque; an aligner handle is bound to one GPU and must be used
 *    from one host thread at a time (the reference's BaseAligner is likewise not
 *    thread safe, Aligner.h:19-20).
 *  - Genome locations are the reference's 0-based offsets into the padded
 *    whole-genome string (Genome.h:29, FASTA.cpp:67-125).
 */
#ifndef SNAPGPU_H
#define SNAPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: snapgpu_timing_t.nNulReads / nUnwritten, SNAPGPU_FLAG_NUL_BYTE, SNAPGPU_PFLAG_NUL_BYTE, the
 *    buffer length of snapgpu_phase_cycles */
#define SNAPGPU_ABI_VERSION 2

enum {
    SNAPGPU_OK = 0,
    SNAPGPU_EINVAL = -1,      /* bad argument */
    SNAPGPU_EIO = -2,         /* file could not be read/written */
    SNAPGPU_ENOMEM = -3,      /* host or device allocation failed */
    SNAPGPU_EDEVICE = -4,     /* HIP runtime error / no GPU */
    SNAPGPU_EFORMAT = -5,     /* index/genome file format error */
    SNAPGPU_EUNSUPPORTED = -6 /* parameter combination not supported */
};

/* AlignmentResult (SNAPLib/Read.h:41) */
enum { SNAPGPU_NOT_FOUND = 0, SNAPGPU_SINGLE_HIT = 1, SNAPGPU_MULTIPLE_HITS = 2, SNAPGPU_UNKNOWN = 3 };
/* Direction (SNAPLib/directions.h:26-35) */
enum { SNAPGPU_FORWARD = 0, SNAPGPU_RC = 1 };

/* per-read flags in snapgpu_result_t.flags */
#define SNAPGPU_FLAG_READ_TOO_LONG  0x01u  /* reference: soft_exit(1), BaseAligner.cpp:609-613 */
#define SNAPGPU_FLAG_MAPQ_FIXED     0x02u  /* MAPQ re-derived on host with libm log10 (boundary case) */
#define SNAPGPU_FLAG_DEFERRED       0x04u  /* left pass 1 (read > 128 bases, or IUPAC codes in both read and
                                              genome): aligned by align_kernel<256> or align_kernel<512> */
#define SNAPGPU_FLAG_TOO_MANY_NS    0x08u  /* countOfNs > maxK (BaseAligner.cpp:652-655) */
#define SNAPGPU_FLAG_BYTE_PATH      0x10u  /* aligned by the byte-compare pass 3, align_kernel<512> (read
                                              > 256 bases, or IUPAC codes in both read and genome) */
#define SNAPGPU_FLAG_NUL_BYTE       0x20u  /* the read holds a 0x00 byte inside its length: no FASTQ/SAM
                                              reader produces one, so it marks a corrupted or unfinished
                                              upload (the aligner still treats it as a non-ACGT base, as
                                              the reference would); counted in snapgpu_timing_t.nNulReads */

/*
 * Result of one AlignRead call (BaseAligner.cpp:510-938).  location / direction /
 * score / mapq are exactly what AlignRead writes through its out-pointers,
 * including the "written before the result is known" conventions
 * (BaseAligner.cpp:582-584, 1357-1360): location=0xffffffff, direction=FORWARD,
 * score=0xffff when nothing was scored.  mapq is 0 when AlignRead returns before
 * writing it (short read / too many Ns).  The remaining fields are the per-read
 * deltas of BaseAligner's statistics getters (BaseAligner.h:113-117) and its
 * private MAPQ inputs (BaseAligner.h:284-285,333), exported for parity checking
 * and roofline accounting.
 */
typedef struct snapgpu_result {
    uint32_t location;
    int32_t  score;
    int32_t  mapq;
    uint8_t  result;      /* SNAPGPU_NOT_FOUND .. */
    uint8_t  direction;   /* SNAPGPU_FORWARD / SNAPGPU_RC */
    uint8_t  flags;       /* SNAPGPU_FLAG_* */
    uint8_t  reserved;
    uint32_t nLookups;            /* getNHashTableLookups() delta */
    uint32_t nLocationsScored;    /* getLocationsScored() delta */
    uint16_t popularSeedsSkipped; /* BaseAligner::popularSeedsSkipped */
    uint16_t nHitsIgnored;        /* getNHitsIgnoredBecauseOfTooHighPopularity() delta */
    uint32_t nProbes;             /* 64-B bucket lines of the seed-table image loaded (roofline P; device statistic) */
    uint32_t nHitWords;           /* hit words consumed (roofline H) */
    uint32_t nOverflowLists;      /* overflow lists visited (roofline V) */
    uint32_t nElements;           /* candidate elements allocated (BaseAligner.cpp:1485-1568) */
    uint32_t reserved2;
    double   probabilityOfAllCandidates;
    double   probabilityOfBestCandidate;
} snapgpu_result_t;   /* 64 bytes */

/* BaseAligner constructor parameters (BaseAligner.h:44-55, defaults of
 * AlignerOptions.cpp:33-85 / SingleAligner.cpp:167-179). */
typedef struct snapgpu_aligner_params {
    uint32_t maxHitsToConsider;  /* -h, default 300 */
    uint32_t maxK;               /* -d, default 14 */
    uint32_t maxReadSize;        /* MAX_READ_LENGTH (Read.h:45), default 500 */
    uint32_t maxSeedsToUse;      /* -n, default 25 (0 => use seedCoverage) */
    double   maxSeedCoverage;    /* -sc, used iff maxSeedsToUse == 0 */
    uint32_t extraSearchDepth;   /* default 2 */
    uint32_t explorePopularSeeds;/* setExplorePopularSeeds (BaseAligner.h:139) */
    uint32_t stopOnFirstHit;     /* setStopOnFirstHit (BaseAligner.h:142) */
} snapgpu_aligner_params_t;

void snapgpu_aligner_params_default(snapgpu_aligner_params_t *p);

/* ------------------------------------------------------------------ genome */
typedef struct snapgpu_genome snapgpu_genome_t;

/* ReadFASTAGenome (SNAPLib/FASTA.cpp:31-130): upper-cases, N -> 'n',
 * `chromosomePadding` 'n's before every contig and at the end. */
snapgpu_genome_t *snapgpu_genome_from_fasta(const char *path, uint32_t chromosomePadding);

/* Deterministic synthetic genome (no reference equivalent; stands in for
 * GRCh38 data that is not available offline).  See DESIGN.md "Synthetic data". */
typedef struct snapgpu_synth_genome_params {
    uint64_t seed;               /* PRNG seed (e.g. 2121) */
    uint64_t totalBases;         /* sum of contig lengths (excl. padding) */
    uint32_t nContigs;
    uint32_t nRepeatFamilies;    /* 0 => uniform random genome */
    double   repeatFraction;     /* target fraction of repeat-derived bases */
    double   maxDivergence;      /* per-copy divergence ~ U(0, maxDivergence) */
    double   nRunFraction;       /* fraction of bases in runs of N */
    uint32_t chromosomePadding;  /* default 500 */
} snapgpu_synth_genome_params_t;
snapgpu_genome_t *snapgpu_genome_synthetic(const snapgpu_synth_genome_params_t *p);
int  snapgpu_genome_write_fasta(const snapgpu_genome_t *g, const char *path);
void snapgpu_genome_free(snapgpu_genome_t *g);
uint32_t snapgpu_genome_nbases(const snapgpu_genome_t *g);
/* pointer to base 0 of the padded genome string; bytes [-256, nBases+256) are readable */
const char *snapgpu_genome_bases(const snapgpu_genome_t *g);
int snapgpu_genome_npieces(const snapgpu_genome_t *g);
uint32_t snapgpu_genome_piece_offset(const snapgpu_genome_t *g, int i);
const char *snapgpu_genome_piece_name(const snapgpu_genome_t *g, int i);

/* ------------------------------------------------------------------- index */
typedef struct snapgpu_index snapgpu_index_t;

/* GenomeIndex::BuildIndexToDirectory semantics (GenomeIndex.cpp:348-720): every
 * genome offset in [0, nBases - seedLen - 1) whose seedLen bases are all ACGT is
 * indexed under its canonical (smaller of seed / reverse complement) seed;
 * overflow lists are sorted descending (GenomeIndex.cpp:616-618).  The layout of
 * the SNAPHashTable slots differs from the reference's multi-threaded builder
 * (as it does between two reference builds), the lookup results do not.
 * Takes ownership of `genome`.  nThreads <= 0 => hardware concurrency. */
snapgpu_index_t *snapgpu_index_build(snapgpu_genome_t *genome, int seedLen, int nThreads);
/* As snapgpu_index_build with the table-size slack of `snap-rna index -h` (GenomeIndex.cpp:208,
 * default 0.3; <= 0 => 0.3): table i gets (nBases * (1 + slack) / nTables) * bias_i slots with the
 * exact bias of ComputeBiasTable (GenomeIndex.cpp:1109-1243, 294-346), at least 100 -- the
 * reference's load factor and probe chains. */
snapgpu_index_t *snapgpu_index_build_ex(snapgpu_genome_t *genome, int seedLen, int nThreads, double slack);
/* GenomeIndex::loadFromDirectory (GenomeIndex.cpp:844-963), reference on-disk format. */
snapgpu_index_t *snapgpu_index_load(const char *directory);
/* Write the reference on-disk format (GenomeIndex.cpp:646-710, Genome.cpp:125-158,
 * HashTable.cpp:180-215) so the reference `snap-rna` can load our index. */
int  snapgpu_index_save(const snapgpu_index_t *idx, const char *directory);
void snapgpu_index_free(snapgpu_index_t *idx);
/* Multi-rank jobs (no reference equivalent: the reference is one process): build the index
 * once per node, write it as one flat file (e.g. under /dev/shm) with snapgpu_index_share, and
 * map it read-only in every rank with snapgpu_index_attach (no private copy of the tables). */
int snapgpu_index_share(const snapgpu_index_t *idx, const char *path);
snapgpu_index_t *snapgpu_index_attach(const char *path);
/* The genome an index owns (valid while the index lives). */
const snapgpu_genome_t *snapgpu_index_genome(const snapgpu_index_t *idx);

typedef struct snapgpu_index_info {
    uint32_t nBases;
    uint32_t seedLen;
    uint32_t nHashTables;
    uint32_t chromosomePadding;
    uint64_t overflowTableSize;   /* u32 words */
    uint64_t totalHashSlots;      /* sum of tableSize */
    uint64_t totalUsedSlots;
    int32_t  nPieces;
    uint32_t hasIupac;            /* genome holds bytes other than ACGTn */
} snapgpu_index_info_t;
int snapgpu_index_get_info(const snapgpu_index_t *idx, snapgpu_index_info_t *info);

/* Raw read-only view of the index tables (SNAPHashTable entries are
 * {u32 key, u32 value1, u32 value2}, HashTable.h:117-123). */
typedef struct snapgpu_index_view {
    const uint32_t *slots;          /* all tables concatenated, 3 words per slot */
    const uint64_t *tableBase;      /* [nHashTables] slot index of table start */
    const uint64_t *tableSize;      /* [nHashTables] */
    const uint32_t *overflow;       /* overflow table (count, hits... descending) */
    const char     *genome;         /* base 0 of padded genome, [-256, nBases+256) readable */
    const uint32_t *pieceOffsets;   /* [nPieces] */
    uint32_t nBases, seedLen, nHashTables, chromosomePadding;
    int32_t  nPieces;
    uint32_t pad_;
    uint64_t overflowTableSize;
} snapgpu_index_view_t;
int snapgpu_index_get_view(const snapgpu_index_t *idx, snapgpu_index_view_t *view);

/* GenomeIndex::lookupSeed (GenomeIndex.cpp:971-1011), host side.  Writes up to
 * `cap` hits per direction; returns the true counts in nHits[2]. */
int snapgpu_index_lookup(const snapgpu_index_t *idx, const char *seedBases,
                         uint32_t nHits[2], uint32_t *hitsFwd, uint32_t *hitsRc, uint32_t cap);

/* ------------------------------------------------------------------- reads */
/* A batch of reads in host memory: read i has bases[offsets[i] .. +lengths[i])
 * and the same range of quals (Phred+33), as Read::getData/getQuality expose
 * them (Read.h:289-328).  Buffers carry >= 16 bytes of zero slack at the end. */
typedef struct snapgpu_reads {
    uint64_t  n;
    uint64_t  totalBytes;
    char     *bases;
    char     *quals;
    uint64_t *offsets;
    uint32_t *lengths;
    uint32_t *truthLocation;   /* generator ground truth (genome offset of read start), or NULL */
    uint8_t  *truthDirection;
    /* Read::clip state (Read.h:357-404), kept by snapgpu_reads_clip: the front clip and the
     * unclipped length of every read (NULL until the first clip), and the clipping applied. */
    uint32_t *frontClipped;
    uint32_t *unclippedLength;
    int32_t   clipping;        /* ReadClippingType last applied (0 = NoClipping) */
    uint32_t  nUploads;        /* device uploads of this batch; clipping is refused after the first */
    /* Read::getId (Read.h:289-328): id i = ids[idOffsets[i] .. +idLengths[i]) (FASTQ header
     * without '@'), or NULL when the batch carries no ids. */
    char     *ids;
    uint64_t *idOffsets;
    uint32_t *idLengths;
    uint32_t  hostFlags;       /* library-internal (bit 0: bases/quals in pinned host memory) */
    uint32_t  reserved_;
} snapgpu_reads_t;

/* wgsim-like simulator: uniform start, 50/50 strand,
 * haplotype mutations (rate, indel fraction) then per-base substitution errors,
 * constant quality char. */
typedef struct snapgpu_synth_reads_params {
    uint64_t seed;              /* e.g. 99 */
    uint64_t nReads;
    uint32_t readLength;        /* 100 */
    uint32_t qualityChar;       /* '2' = Q17, as wgsim writes for 2% error */
    double   baseErrorRate;     /* 0.02 */
    double   mutationRate;      /* 0.001 */
    double   indelFraction;     /* 0.15 */
    double   indelExtend;       /* 0.3 */
    double   randomReadFraction;/* fraction of reads of pure noise (NotFound) */
} snapgpu_synth_reads_params_t;
snapgpu_reads_t *snapgpu_reads_synthetic(const snapgpu_genome_t *g, const snapgpu_synth_reads_params_t *p);
/* wgsim-like read pairs (nReads pairs, readLength each): insert ~ N(insertMean, insertSd). */
int snapgpu_reads_synthetic_pairs(const snapgpu_genome_t *g, const snapgpu_synth_reads_params_t *p, uint32_t insertMean,
                                  uint32_t insertSd, snapgpu_reads_t **reads0, snapgpu_reads_t **reads1);
snapgpu_reads_t *snapgpu_reads_from_fastq(const char *path);
/* Build a batch from caller arrays (copies them). */
snapgpu_reads_t *snapgpu_reads_from_arrays(uint64_t n, const char *bases, const char *quals,
                                           const uint64_t *offsets, const uint32_t *lengths);
int  snapgpu_reads_write_fastq(const snapgpu_reads_t *r, const char *path);
void snapgpu_reads_free(snapgpu_reads_t *r);

/* ----------------------------------------------------------------- aligner */
typedef struct snapgpu_aligner snapgpu_aligner_t;

int  snapgpu_device_count(void);
int  snapgpu_device_cu_count(int device);   /* compute units of a device (0 if none) */
/* BaseAligner::BaseAligner (BaseAligner.cpp:46-194) + index upload to HBM.  The
 * index must outlive the aligner. */
snapgpu_aligner_t *snapgpu_aligner_create(int device, const snapgpu_index_t *idx,
                                          const snapgpu_aligner_params_t *params);
void snapgpu_aligner_free(snapgpu_aligner_t *a);

/* Batched BaseAligner::AlignRead (BaseAligner.cpp:196-200 / 510-938) over host
 * buffers: H2D of the reads, the GPU passes, D2H of the records. */
int snapgpu_align_batch(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, snapgpu_result_t *out);

/* Streaming form of snapgpu_align_batch for callers that keep several batches in flight (the
 * GpuSingleExtension pattern): submit returns once the batch is queued (its last chunks still
 * on the GPU; earlier batches' chunks are finished as their streams are reused); wait drains
 * everything submitted.  reads and out must stay valid, and out untouched, until the wait.
 * snapgpu_last_timing then covers every batch since the previous wait. */
int snapgpu_align_batch_submit(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, snapgpu_result_t *out);
int snapgpu_align_batch_wait(snapgpu_aligner_t *a);

/* The extended AlignRead (BaseAligner.h:72-86, BaseAligner.cpp:510-938) used by the
 * paired / transcriptome callers:
 *  - per-read search window: searchRadius != 0 restricts hits to genome locations
 *    within searchRadius of searchLocation, in searchDirection only (windowed
 *    GenomeIndex::lookupSeed, GenomeIndex.cpp:1013-1086, and BaseAligner.cpp:781-853);
 *  - multi-hit export (fillHitsFound, BaseAligner.cpp:940-975, recording at :1255-1261):
 *    up to maxHitsToGet hits with edit distance in [best, best+3] per read, written to
 *    multiHits[i * maxHitsToGet ..], their count to multiHitsFound[i]; entries past
 *    multiHitsFound[i] in a read's row are left untouched (only the found hits are copied
 *    back, compacted on the device).
 * search may be NULL (no window for any read); maxHitsToGet 0 disables multi-hit
 * export (multiHitsFound / multiHits may then be NULL); at most SNAPGPU_MAX_MULTI_HITS_TO_GET.
 * The reference keeps 512 hits per distance (BaseAligner.h:148-151) but counts up to
 * maxHitsToGet per distance, so above 512 a distance's extra hits overwrite the next
 * distances' rows; that layout is reproduced (the RNA paired path asks for 1000,
 * PairedAligner.cpp:584).  maxHitsToGet > 512 needs (maxK + extraSearchDepth) * 512 +
 * maxHitsToGet <= 31 * 512 (the writes stay inside the reference's table). */
#define SNAPGPU_MAX_MULTI_HITS_TO_GET 1024
typedef struct snapgpu_search {
    uint32_t searchRadius;
    uint32_t searchLocation;
    uint32_t searchDirection;   /* SNAPGPU_FORWARD / SNAPGPU_RC */
    uint32_t reserved;
} snapgpu_search_t;
typedef struct snapgpu_multi_hit {
    uint32_t location;
    uint8_t  direction;         /* multiHitRCs */
    uint8_t  score;             /* multiHitScores */
    uint16_t reserved;
} snapgpu_multi_hit_t;
int snapgpu_align_batch_ex(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, const snapgpu_search_t *search,
                           uint32_t maxHitsToGet, snapgpu_result_t *out, int32_t *multiHitsFound,
                           snapgpu_multi_hit_t *multiHits);

/* Device-resident variant: reads are uploaded once with snapgpu_reads_upload;
 * snapgpu_align_resident runs only the GPU passes (inputs already in HBM, output
 * left in HBM); snapgpu_results_download copies the records back. */
typedef struct snapgpu_device_reads snapgpu_device_reads_t;
snapgpu_device_reads_t *snapgpu_reads_upload(snapgpu_aligner_t *a, const snapgpu_reads_t *reads);
void snapgpu_device_reads_free(snapgpu_device_reads_t *d);
int  snapgpu_align_resident(snapgpu_aligner_t *a, snapgpu_device_reads_t *d);
int  snapgpu_results_download(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, snapgpu_result_t *out);
int  snapgpu_synchronize(snapgpu_aligner_t *a);

/* Timing of the dominant kernel (HIP events on the stream it ran on), in ms, for the last
 * snapgpu_align_resident / snapgpu_align_batch call.  snapgpu_align_batch pipelines its reads
 * in chunks over two streams: the kernel figures are then sums over its nLaunches chunks. */
typedef struct snapgpu_timing {
    double mainKernelMs;     /* pass 1: align_kernel<128> (reads <= 128 bases, bit-plane LV) */
    double spillKernelMs;    /* passes 2 + 3: align_kernel<256> over the reads pass 1 deferred
                                (129..256 bases, bit-plane LV), align_kernel<512> over the rest */
    double fixupMs;          /* host MAPQ fix-ups */
    uint64_t nSpilled;       /* reads deferred by pass 1 */
    uint64_t nMapqFixed;
    double lookupKernelMs;   /* pass 0: seed_lookup_kernel (first-round seed lookups) */
    uint64_t lookupSeeds;    /* seeds it looked up */
    uint64_t lookupProbes;   /* bucket lines it loaded */
    uint64_t lookupOverflowReads; /* overflow-list counts it read */
    uint64_t nLaunches;      /* pass sets the figures above sum over (chunks of snapgpu_align_batch) */
    double wallMs;           /* snapgpu_align_batch: host reads in -> records out, whole call */
    double mainKernelBusyMs; /* union of the pass-1 launch intervals (launches of the two lanes overlap) */
    double lookupKernelBusyMs;/* union of the pass-0 launch intervals */
    uint64_t nByteReads;     /* reads deferred by pass 2 to the byte-compare pass 3 (> 256 bases,
                                or IUPAC codes in both read and genome) */
    uint64_t nArenaOverflow; /* reads that outgrew a capped element arena in passes 1-3 and were
                                aligned again by the big-arena pass (worst-case arenas, small grid) */
    uint64_t nNulReads;      /* records with SNAPGPU_FLAG_NUL_BYTE (0 for any FASTQ input) */
    uint64_t nUnwritten;     /* records no pass wrote (the device output is pre-filled with 0xff
                                and every read must get exactly one record): always 0, else the
                                call fails with SNAPGPU_EDEVICE */
} snapgpu_timing_t;
int snapgpu_last_timing(snapgpu_aligner_t *a, snapgpu_timing_t *t);

/* Aggregated getters of the reference aligner (Aligner.h:62-70). */
typedef struct snapgpu_aligner_stats {
    int64_t nHashTableLookups;
    int64_t nLocationsScored;
    int64_t nHitsIgnoredBecauseOfTooHighPopularity;
    int64_t nReadsIgnoredBecauseOfTooManyNs;
    int64_t nIndelsMerged;
    int64_t nReads;
} snapgpu_aligner_stats_t;
int snapgpu_aligner_get_stats(const snapgpu_aligner_t *a, snapgpu_aligner_stats_t *s);
int snapgpu_aligner_max_k(const snapgpu_aligner_t *a);           /* getMaxK() */
/* Whether the pass sets of the aligner's two streams may run concurrently (default 1; the
 * environment variable SNAPGPU_OVERLAP sets the initial value).  0 serialises the kernels
 * (copies and host work still overlap them): each launch's duration is then its own. */
int snapgpu_aligner_set_overlap(snapgpu_aligner_t *a, int overlap);
/* Test hook (no reference equivalent): the aligner's next calls trip its device watchdog when
 * the batch's read `read_index` starts (0xffffffff: never), so the call fails with
 * SNAPGPU_EDEVICE.  Each aligner has its own watchdog record: a trip in one aligner neither
 * fails nor stops another aligner on the same device. */
int snapgpu_aligner_debug_trip(snapgpu_aligner_t *a, uint32_t read_index);
/* SHA-256 of the sources this library was built from (snapgpu/_srcsha.py: csrc, this header, the
 * Makefile); the Python loader refuses a library whose identity differs from the sources beside it. */
const char *snapgpu_source_sha256(void);
/* Diagnostic (no reference equivalent): with SNAPGPU_PHASES=1 in the environment at
 * snapgpu_aligner_create, align_kernel<128> sums shader cycles per phase and event
 * counts into out[0..min(len, 48)) (order: snapgpu.BaseAligner.PHASES); reset != 0 zeroes them. */
int snapgpu_phase_cycles(snapgpu_aligner_t *a, uint64_t *out, uint32_t len, int reset);
const char *snapgpu_aligner_name(const snapgpu_aligner_t *a);    /* getName() */

/* -------------------------------------------------------- Landau-Vishkin */
/* LandauVishkin<dir>::computeEditDistance (LandauVishkin.h:211-455) on the GPU,
 * one call per task, for unit parity (reference tests/LandauVishkinTest.cpp).
 * Task i: text = texts[textOff[i] .. +textLen[i]) (for dir=-1 the text is
 * walked backwards from its last byte, as a reverse LV called with a pointer
 * one past the end), pattern/quals = patterns/quals[patOff[i] .. +patLen[i]).
 * Out: edit distance or -1, netIndel, matchProbability. */
int snapgpu_lv_batch(int device, int direction, uint32_t n,
                     const char *texts, const uint64_t *textOff, const uint32_t *textLen,
                     const char *patterns, const char *quals, const uint64_t *patOff,
                     const uint32_t *patLen, const int32_t *k,
                     int32_t *outScore, int32_t *outNetIndel, double *outProb);

/* The same calls through the production bit-plane LV of align_kernel<128> / <256> (lv_group /
 * lv_prob_pair in align_score.h) instead of the byte-compare engine: unit parity for the LV
 * that scores every read of <= 256 bases.  Patterns of 1..253 bases: a batch whose patterns
 * are all <= 127 runs on 128-bit masks (align_kernel<128>), any longer pattern puts the whole
 * batch on 256-bit masks (align_kernel<256>); netIndel is reported for direction -1 only
 * (the aligner uses only the reverse call's, BaseAligner.cpp:1232). */
int snapgpu_lv_group_batch(int device, int direction, uint32_t n,
                           const char *texts, const uint64_t *textOff, const uint32_t *textLen,
                           const char *patterns, const char *quals, const uint64_t *patOff,
                           const uint32_t *patLen, const int32_t *k,
                           int32_t *outScore, int32_t *outNetIndel, double *outProb);

/* ------------------------------------------------- CIGAR / SAM records */
/* The SAM writer's per-read work, on the GPU:
 * LandauVishkinWithCigar::computeEditDistance (LandauVishkin.cpp:252-535) as
 * SAMFormat::computeCigarString (SAM.cpp:1162-1230) calls it -- text = the genome
 * substring at the location with the read's length, k = MAX_K - 1, the read
 * upper-cased and, for RC, reverse-complemented (getSAMData, SAM.cpp:866-883).
 * Per read out: editDistance (the NM tag; -1 when the reference prints "*": no
 * location, no substring (Genome::getSubstring NULL) or no alignment within k),
 * nOps, and ops[i * SNAPGPU_CIGAR_MAX_OPS ..] as BAM ops (count << 4 | code, code
 * index into "MIDNSHP=X"; useM != 0 is the `-M` form: '=' and 'X' merged into 'M').
 * snapgpu_cigar_batch writes the first nOps[i] entries of row i only.
 * Reads longer than 512 bases are rejected (SNAPGPU_EINVAL). */
#define SNAPGPU_CIGAR_MAX_OPS 64

/* Explicit (location, direction) per read; location 0xffffffff => "*". */
int snapgpu_cigar_batch(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, const uint32_t *locations,
                        const uint8_t *directions, int useM, int32_t *editDistance, uint32_t *nOps, uint32_t *ops);
/* Device-resident: the CIGARs of the records the last snapgpu_align_resident left
 * in HBM for these reads, with writeRead's rules (SAM.cpp:1007-1048, 855-883): a
 * NotFound record keeps its location for the CIGAR but uses the forward read. */
int snapgpu_cigar_resident(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, int useM);
int snapgpu_cigar_download(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, int32_t *editDistance, uint32_t *nOps,
                           uint32_t *ops);
/* cigar_kernel time of the last snapgpu_cigar_resident / snapgpu_cigar_batch (HIP events). */
int snapgpu_cigar_last_ms(snapgpu_aligner_t *a, double *ms);

/* One SAM line per read, as SAMFormat::writeRead (SAM.cpp:1007-1155) writes it for a
 * single-end genome alignment: QNAME (read id up to the first space), FLAG, RNAME,
 * POS, MAPQ (clamped to [0, 70]; 0 when unmapped), CIGAR, "*", 0, 0, SEQ and QUAL
 * (reverse-complemented / reversed for RC), RG:Z:<readGroup> (omitted when NULL),
 * PG:Z:SNAP, NM:i:<editDistance>.  ids[idOffsets[i] .. +idLengths[i]) is read i's
 * id.  Writes at most `cap` bytes to out and the size needed to *used; returns
 * SNAPGPU_EINVAL (nothing usable written) when cap is too small. */
int snapgpu_sam_format(const snapgpu_index_t *idx, const snapgpu_reads_t *reads, const char *ids,
                       const uint64_t *idOffsets, const uint32_t *idLengths, const snapgpu_result_t *results,
                       const int32_t *editDistance, const uint32_t *nOps, const uint32_t *ops,
                       const char *readGroup, char *out, uint64_t cap, uint64_t *used);

/* Clipped reads (Read::clip, Read.h:357-404, applied by the FASTQ reader, FASTQ.cpp:250;
 * clipping = NoClipping 0 / ClipFront 1 / ClipBack 2 / ClipFrontAndBack 3 -- the reference's
 * default is 3): snapgpu_reads_clip narrows offsets/lengths in place to the clipped read (what
 * the aligner and the CIGAR kernel see) and returns the front clip and unclipped length per
 * read; snapgpu_sam_format_clipped then prints the unclipped SEQ/QUAL and the soft clips
 * ("%uS" before / after the CIGAR, mirrored for RC -- SAM.cpp:866-883, 1212-1226). */
int snapgpu_reads_clip(snapgpu_reads_t *reads, int clipping, uint32_t *frontClipped, uint32_t *unclippedLength);
int snapgpu_sam_format_clipped(const snapgpu_index_t *idx, const snapgpu_reads_t *reads, const char *ids,
                               const uint64_t *idOffsets, const uint32_t *idLengths, const snapgpu_result_t *results,
                               const int32_t *editDistance, const uint32_t *nOps, const uint32_t *ops,
                               const char *readGroup, const uint32_t *frontClipped, const uint32_t *unclippedLength,
                               char *out, uint64_t cap, uint64_t *used);

/* The SAM header as SAMFormat::writeHeader (SAM.cpp:700-800) writes it for a FASTQ input:
 * @HD (SO:coordinate if sorted), rgLine or "@RG\tID:FASTQ\tSM:sample", @PG with CL:commandLine
 * and VN:version, one @SQ per genome piece.  Same size / error contract as snapgpu_sam_format. */
int snapgpu_sam_header(const snapgpu_index_t *idx, int sorted, const char *commandLine, const char *version,
                       const char *rgLine, char *out, uint64_t cap, uint64_t *used);

/* --------------------------------------------- RNA annotation (GTF) */
/* GTFReader (SNAPLib/GTFReader.cpp): exon lines of a GTF/GFF3 file -> transcripts, each an
 * exon list sorted by start with an intron feature between consecutive exons (Load :1245,
 * Parse :1302, GTFTranscript::Process :972). */
typedef struct snapgpu_gtf snapgpu_gtf_t;
snapgpu_gtf_t *snapgpu_gtf_load(const char *path);
void snapgpu_gtf_free(snapgpu_gtf_t *gtf);
int snapgpu_gtf_counts(const snapgpu_gtf_t *gtf, uint32_t *nFeatures, uint32_t *nTranscripts, uint32_t *nGenes);
/* GTFReader::BuildTranscriptome (GTFReader.cpp:1840-1867): the FASTA `snap-rna transcriptome`
 * indexes -- every transcript (id order) as the genome bytes of its exon/intron list. */
int snapgpu_gtf_write_transcriptome(const snapgpu_gtf_t *gtf, const snapgpu_genome_t *genome, const char *fastaPath);
/* GTFTranscript::GenomicPosition (GTFReader.cpp:1075-1105): 1-based transcript position ->
 * 1-based genomic position (0 when the span runs past the transcript). */
int snapgpu_gtf_genomic_position(const snapgpu_gtf_t *gtf, const char *transcriptId, uint32_t pos, uint32_t span,
                                 uint32_t *genomicPos);
/* LandauVishkinWithCigar::insertSpliceJunctions (LandauVishkin.cpp:119-250): the CIGAR of a
 * transcriptome alignment at 1-based transcript position `pos`, given as (count, op) tokens,
 * with 'N' runs inserted at the transcript's junctions.  NUL-terminated string out. */
int snapgpu_gtf_splice_cigar(const snapgpu_gtf_t *gtf, const char *transcriptId, uint32_t pos, uint32_t nTokens,
                             const uint32_t *counts, const char *ops, char *out, uint64_t cap, uint64_t *used);

/* ----------------------------------- single-end product path (f1) */
/* SingleAlignerContext::runIterationThread (SNAPLib/SingleAligner.cpp:141-320) batched on the
 * GPU: per read Read::clip, the quality / length / N pre-filter (:247-257), the transcriptome
 * and genome BaseAligner::AlignRead (two aligners, :270-276), AlignmentFilter::AddAlignment /
 * FilterSingle (AlignmentFilter.cpp:140-300) and SAMFormat::writeRead (SAM.cpp:978-1153:
 * GPU CIGARs, transcriptome records with insertSpliceJunctions) -- the SAM file `snap-rna single
 * <genome> <transcriptome> <gtf> <reads>` writes, and the gene read counts FilterSingle records
 * (snapgpu_gtf_write_counts writes the count files).  Not built: the contamination database (-x),
 * BAM / sorted output. */
typedef struct snapgpu_single_options {
    int32_t  clipping;               /* ReadClippingType, default 3 = ClipFrontAndBack (AlignerOptions.cpp:48) */
    uint32_t confDiff;               /* -c, default 2 */
    uint32_t maxDist;                /* -d, default 14 (the filter's maxDist) */
    float    minPercentAbovePhred;   /* -fp, default 90 */
    uint32_t minPhred;               /* -fm, default 20 */
    uint32_t phredOffset;            /* -fo, default 33 */
    uint32_t useM;                   /* -M */
    uint32_t sortOutput;             /* -so: SAM records stable-sorted by location, @HD SO:coordinate
                                        (SortedDataWriter.cpp:186-240; one block per call; not for BAM) */
    const char *readGroup;           /* default "FASTQ" (AlignerOptions.cpp:65) */
    const char *commandLine;         /* @PG CL: */
    const char *version;             /* @PG VN: */
    /* -ct: the contamination database (SingleAligner.cpp:205-218, 282-293): reads the filter left
     * NotFound go through this BaseAligner (same parameters as the genome aligner) and each one it
     * aligns is counted in `contaminants` (both NULL: no contamination database) */
    struct snapgpu_aligner *contaminationAligner;
    struct snapgpu_contaminants *contaminants;
} snapgpu_single_options_t;
void snapgpu_single_options_default(snapgpu_single_options_t *o);

typedef struct snapgpu_single_stats {   /* AlignerStats (AlignerStats.h:40-69) */
    uint64_t totalReads, usefulReads, singleHits, multiHits, notFound, transcriptomeRecords;
    double alignMs, cigarMs, filterMs, writeMs, wallMs;
    double prepMs;   /* clipping, pre-filter, the batch view and the per-read arrays (before alignMs) */
    double formatMs, ioMs;   /* of writeMs: the records' text (host threads), the file output */
} snapgpu_single_stats_t;

/* reads: a FASTQ batch with ids (snapgpu_reads_from_fastq), clipped here.  samPath receives
 * the header and one record per read in input order: SAM text, or BGZF-compressed BAM when the
 * path ends in ".bam" (BAMFormat::writeHeader / writeRead, Bam.cpp:542-790). */
int snapgpu_single_align(snapgpu_aligner_t *genomeAligner, snapgpu_aligner_t *transcriptomeAligner,
                         snapgpu_gtf_t *gtf, snapgpu_reads_t *reads, const snapgpu_single_options_t *opt,
                         const char *samPath, snapgpu_single_stats_t *stats);
/* `-so` for SAM text (SortedDataFilter::onNextBatch, SortedDataWriter.cpp:186-240): the records
 * (lines) of `in` stable-sorted by SAMFormat::getSortInfo's location (SAM.cpp:639-685) over idx's
 * genome; header lines (starting '@') are not records and must not be in `in`.  Writes at most cap
 * bytes to out, *used = the size (= n); the product paths use it with sortOutput set. */
int snapgpu_sam_sort_records(const snapgpu_index_t *idx, const char *in, uint64_t n, char *out, uint64_t cap,
                             uint64_t *used);

/* ------------------------------------------ contamination database (-ct) counts */
/* ContaminationFilter (ContaminationFilter.cpp:22-112): contaminant alignments counted per contig
 * of the contamination genome (a location maps to its piece, Genome::getPieceAtLocation; an
 * invalid location counts nothing).  Counts accumulate over the product-path calls that carry the
 * object in their options; thread-safe. */
typedef struct snapgpu_contaminants snapgpu_contaminants_t;
snapgpu_contaminants_t *snapgpu_contaminants_create(const snapgpu_index_t *contamination);
void snapgpu_contaminants_free(snapgpu_contaminants_t *c);
int snapgpu_contaminants_add(snapgpu_contaminants_t *c, uint32_t location);   /* AddAlignment */
/* ContaminationFilter::Write: "<prefix>.contaminants.txt" with prefix = outputFileTemplate up to
 * its last '.' ("default" for NULL), one "contig<TAB>count" line per contig, by count descending
 * (the reference's std::sort over the name-ordered counts, reverse iterators) */
int snapgpu_contaminants_write(const snapgpu_contaminants_t *c, const char *outputFileTemplate);
/* the same text into out (at most cap bytes; *used = the size needed) */
int snapgpu_contaminants_format(const snapgpu_contaminants_t *c, char *out, uint64_t cap, uint64_t *used);

/* The index an aligner was created over (BaseAligner's GenomeIndex; getGenome for the SAM writer). */
const snapgpu_index_t *snapgpu_aligner_index(const snapgpu_aligner_t *a);
int snapgpu_aligner_get_params(const snapgpu_aligner_t *a, snapgpu_aligner_params_t *p);

/* Roofline calibration (diagnostic, no reference equivalent): time of nLoads independent
 * 64-byte bucket-line loads at hashed positions of this aligner's resident bucket image
 * (the access pattern of the seed lookups without their dependency chain), best of 3, ms. */
int snapgpu_gather_peak(snapgpu_aligner_t *a, uint32_t nLoads, double *ms);

/* The device image of the seed tables (no reference equivalent: SNAPHashTable's key -> value map
 * re-laid into 64-byte buckets of four {key, value1, value2, counts} entries when the aligner is
 * created; GenomeIndex::lookupSeed answers are unchanged).  Diagnostic figures of that image. */
typedef struct snapgpu_bucket_info {
    uint64_t nSlots;            /* reference-format slots the image was built from */
    uint64_t nKeys;             /* keys it holds (slots SNAPHashTable::Lookup can return) */
    uint64_t nBuckets;          /* 64-byte buckets */
    uint64_t nOverflowBuckets;  /* buckets flagged: a key homed there lives in a later bucket */
    uint64_t maxDisplacement;   /* most buckets a key lives past its home */
    uint64_t bytes;             /* HBM of the image */
    double buildMs;             /* slots upload + count + build, wall */
} snapgpu_bucket_info_t;
int snapgpu_aligner_bucket_info(const snapgpu_aligner_t *a, snapgpu_bucket_info_t *info);
/* GenomeIndex::lookupSeed + fillInLookedUpResults (GenomeIndex.cpp:971-1086, unwindowed) of n seeds
 * (seedLen ACGT bases each, concatenated) on the device, through the bucket image: mode 0 = one lane
 * per seed, each lane loading its whole line (bucket_lookup_lane: the paired kernel's lookup), 1 = the
 * whole wave per seed (bucket_lookup_wave: the aligner's and CharacterizeSeeds' in-kernel lookups),
 * 2 = one lane per seed, four lanes per line (bucket_lookup_quad: seed_lookup_kernel's lookup), run
 * on waves with a scattered half of their lanes active.  out[6 i ..]: hits forward, hits RC,
 * hash of the forward hits, of the RC hits (acc = acc * 1000003 + hit, list order, mod 2^64),
 * first forward hit, first RC hit (~0 when none); lines[i] = bucket lines loaded. */
int snapgpu_aligner_lookup_seeds(snapgpu_aligner_t *a, const char *seedBases, uint64_t n, int mode, uint64_t *out,
                                 uint32_t *lines);

/* HBM streaming-copy ceiling (diagnostic): best-of-3 time (ms) of copy_peak_kernel reading
 * `bytes` and writing `bytes` with 16-byte vector accesses. */
int snapgpu_copy_peak(snapgpu_aligner_t *a, uint64_t bytes, double *ms);

/* Self-test of the device-timeout path (diagnostic, needs no GPU): a wait that times out must
 * fail with SNAPGPU_EDEVICE, mark the aligner failed, and free no device buffer afterwards.
 * Returns 0 when the path behaves. */
int snapgpu_selftest_timeout_path(void);

/* ------------------------------------------------------------------ paired-end
 * ChimericPairedEndAligner::align (ChimericPairedEndAligner.cpp:56-126) over
 * IntersectingPairedEndAligner::align (IntersectingPairedEndAligner.cpp:142-753), constructed as
 * PairedAligner.cpp:462-482 does.  Defaults = the paired CLI's (AlignerOptions.cpp:73-77,
 * PairedAligner.cpp:57-58, 231-235, IntersectingPairedEndAligner.h:32-33). */
typedef struct snapgpu_paired_params {
    uint32_t maxHits;              /* -h: maxHits of the chimeric single-end fallback, default 16000 */
    uint32_t maxK;                 /* -d: maxDist, default 15 */
    uint32_t maxSeedsToUse;        /* -n: default 8 (0 => seedCoverage) */
    uint32_t extraSearchDepth;     /* default 2 */
    uint32_t minSpacing;           /* -s min, default 50 */
    uint32_t maxSpacing;           /* -s max, default 1000 */
    uint32_t maxBigHits;           /* -H intersectingAlignerMaxHits, default 16000 */
    uint32_t maxCandidatePoolSize; /* -mcp, default 1000000 */
    uint32_t maxReadSize;          /* MAX_READ_LENGTH (Read.h:45), default 500 */
    uint32_t forceSpacing;         /* -f, default 0 */
    double   seedCoverage;         /* used iff maxSeedsToUse == 0 */
} snapgpu_paired_params_t;

/* PairedAlignmentResult (PairedEndAligner.h:31-55) plus counters.  Fields an aligner leaves
 * unwritten keep the pre-state {status NotFound, location 0xffffffff, direction 0, score -1, mapq 0}. */
typedef struct snapgpu_pair_result {
    uint32_t location[2];
    int32_t  score[2];
    int32_t  mapq[2];
    uint8_t  status[2];            /* SNAPGPU_NOT_FOUND .. */
    uint8_t  direction[2];
    uint8_t  fromAlignTogether;
    uint8_t  alignedAsPair;
    uint16_t flags;                /* SNAPGPU_PFLAG_* */
    uint32_t nLocationsScored;     /* IntersectingPairedEndAligner::getLocationsScored() delta */
    uint32_t nSingleScored;        /* the fallback BaseAligner's getLocationsScored() delta */
    uint32_t popularSeedsSkipped;  /* both reads' popular seeds (the MAPQ input, :741) */
    uint32_t writtenBy;            /* routing (diagnostic): the intersecting pass that wrote the record --
                                      1 pass 1 (<128>), 2 pass 1b (<256>), 3 pass 2 (<512>), 4 pass 3
                                      (the reference's pools); 0 for a pair whose mates are both < 50 */
    double   probabilityOfAllPairs;   /* the intersecting aligner's MAPQ inputs (align()'s locals) */
    double   probabilityOfBestPair;
} snapgpu_pair_result_t;   /* 64 bytes */
#define SNAPGPU_PFLAG_POOL_EXHAUSTED 0x01   /* the reference soft_exits ("Ran out of ... pool entries") */
#define SNAPGPU_PFLAG_READ_TOO_LONG  0x02   /* the reference soft_exits (IntersectingPairedEndAligner.cpp:211-215) */
#define SNAPGPU_PFLAG_DEFERRED       0x04   /* left pass 1: aligned by the long-read pass or the large-pool pass */
#define SNAPGPU_PFLAG_MAPQ_FIXED     0x08   /* MAPQ re-derived on the host (threshold case) */
#define SNAPGPU_PFLAG_NUL_BYTE       0x10   /* a read of the pair holds a 0x00 byte inside its length (a
                                               corrupted upload; see SNAPGPU_FLAG_NUL_BYTE) */

void snapgpu_paired_params_default(snapgpu_paired_params_t *p);
typedef struct snapgpu_paired_aligner snapgpu_paired_aligner_t;
/* NULL (and snapgpu_last_error) without a HIP device: there is no CPU fallback. */
snapgpu_paired_aligner_t *snapgpu_paired_aligner_create(int device, const snapgpu_index_t *idx,
                                                        const snapgpu_paired_params_t *p);
void snapgpu_paired_aligner_free(snapgpu_paired_aligner_t *pa);
/* ChimericPairedEndAligner::align for pair i = (reads0[i], reads1[i]), every i, in order. */
int snapgpu_paired_align_batch(snapgpu_paired_aligner_t *pa, const snapgpu_reads_t *reads0,
                               const snapgpu_reads_t *reads1, snapgpu_pair_result_t *out);
/* IntersectingPairedEndAligner::align alone (no single-end fallback), for parity tests. */
int snapgpu_paired_intersect_batch(snapgpu_paired_aligner_t *pa, const snapgpu_reads_t *reads0,
                                   const snapgpu_reads_t *reads1, snapgpu_pair_result_t *out);
/* The single-end BaseAligner the chimeric fallback uses (maxHits, maxK, seeds of the params). */
snapgpu_aligner_t *snapgpu_paired_aligner_single(snapgpu_paired_aligner_t *pa);

/* ------------------------------------------- RNA seed census
 * BaseAligner::CharacterizeSeeds (BaseAligner.cpp:206-508) on the GPU: the seeds of AlignRead's
 * order until numSeeds directions applied (or the wrap runs out), every hit of a side that is
 * not popular recorded as (read-start location implied by the hit, seed offset).  The
 * reference returns two std::map<unsigned, std::set<unsigned>> (map = forward, mapRC = RC);
 * here each map entry is one run record, forward runs first, then RC runs, locations ascending
 * (the maps' iteration order).  The caller's aligner supplies the index (its HBM upload); the
 * scan parameters are those of the partial aligner PairedAligner.cpp:518-527 constructs. */
typedef struct snapgpu_seed_run {
    uint32_t location;     /* map key */
    uint16_t minOffset;    /* *set.begin(): smallest seed offset (forward-read coordinates) */
    uint16_t maxOffset;    /* *set.rbegin() */
    uint16_t count;        /* set.size() */
    uint8_t  direction;    /* 0: map, 1: mapRC */
    uint8_t  reserved;
} snapgpu_seed_run_t;      /* 12 bytes */
typedef struct snapgpu_seed_runs {
    uint64_t n;                 /* reads scanned */
    uint64_t *start;            /* [n + 1]: read i's runs are runs[start[i] .. start[i + 1]) */
    uint32_t *nForward;         /* [n]: how many of them are forward (map) runs */
    uint32_t *flags;            /* [n]: SNAPGPU_FLAG_READ_TOO_LONG (the reference exits), SNAPGPU_FLAG_TOO_MANY_NS */
    snapgpu_seed_run_t *runs;
    uint64_t nRuns;
} snapgpu_seed_runs_t;
typedef struct snapgpu_charseeds_params {
    uint32_t maxHits;              /* 300 (PairedAligner.cpp:520) */
    uint32_t maxK;                 /* the paired maxDist, 15: reads with more Ns are skipped */
    uint32_t numSeeds;             /* 12 (PairedAligner.cpp:523) */
    uint32_t maxReadSize;          /* 500 */
    uint32_t explorePopularSeeds;  /* 0 */
    uint32_t reserved;
} snapgpu_charseeds_params_t;
void snapgpu_charseeds_params_default(snapgpu_charseeds_params_t *p);
/* readList: indices into reads of the reads to scan (NULL: all, nList ignored).  Needs
 * (numSeeds + 1) * maxHits <= 4096 and maxReadSize <= 512.  NULL on error (snapgpu_last_error). */
snapgpu_seed_runs_t *snapgpu_characterize_seeds(snapgpu_aligner_t *a, const snapgpu_reads_t *reads,
                                                const uint64_t *readList, uint64_t nList,
                                                const snapgpu_charseeds_params_t *p);
void snapgpu_seed_runs_free(snapgpu_seed_runs_t *runs);

/* --------------------------------------- RNA paired-end product path
 * PairedAlignerContext::runIterationThread (SNAPLib/PairedAligner.cpp:405-689) batched on the
 * GPU -- what `snap-rna paired <genome> <transcriptome> <gtf> r1.fq r2.fq` computes per pair:
 * Read::clip, the length / N / quality pre-filter (:555-575), transcriptome AlignRead of each
 * read with 1000-hit export (:584-614), the genome ChimericPairedEndAligner (:625),
 * AlignmentFilter::AddAlignment / Filter (AlignmentFilter.cpp:140-214, 302-739) with
 * FindPartialMatches' CharacterizeSeeds on the GPU (:957-1037), forceSpacing and the MAPQ
 * halving (:648-663), the SAM pair records (ReadWriter.cpp:133-217, SAM.cpp:804-1153: GPU
 * CIGARs, insertSpliceJunctions for transcriptome records) and the GTF read counts
 * (GTFReader::IncrementReadCount, GTFReader.cpp:1409-1611; snapgpu_gtf_write_counts writes
 * them).  Not built: the contamination database (-x) and GTFReader::AnalyzeReadIntervals
 * (the interval report UnalignedRead and the *chromosomalPair calls feed). */
typedef struct snapgpu_rna_paired_options {
    int32_t  clipping;               /* ReadClippingType, default 3 (AlignerOptions.cpp:48) */
    uint32_t confDiff;               /* -c, default 2 */
    uint32_t maxDist;                /* -d, default 15 (filter cut-off and the partial aligner's maxK) */
    uint32_t minSpacing, maxSpacing; /* -s, default 50 1000 */
    uint32_t forceSpacing;           /* -fs */
    float    minPercentAbovePhred;   /* -fp, default 90 */
    uint32_t minPhred;               /* -fm, default 20 */
    uint32_t phredOffset;            /* -fo, default 33 */
    uint32_t useM;                   /* -M */
    uint32_t maxHitsToGet;           /* transcriptome multi-hits per read, 1000 (PairedAligner.cpp:584) */
    uint32_t ignoreMismatchedIDs;    /* -I (else mismatched ids fail the call: the reference exits) */
    const char *readGroup;           /* default "FASTQ" */
    const char *commandLine;         /* @PG CL: */
    const char *version;             /* @PG VN: */
    /* -ct: the contamination database (PairedAligner.cpp:487-505, 632-645): pairs the filter left
     * NotFound on both ends go through this paired aligner (the genome one's parameters); a pair
     * it aligns on both ends adds both ends to `contaminants` (both NULL: none) */
    struct snapgpu_paired_aligner *contaminationAligner;
    struct snapgpu_contaminants *contaminants;
    uint32_t sortOutput;             /* -so: as snapgpu_single_options_t.sortOutput */
} snapgpu_rna_paired_options_t;
void snapgpu_rna_paired_options_default(snapgpu_rna_paired_options_t *o);

typedef struct snapgpu_rna_pair_result {   /* PairedAlignmentResult after the filter (PairedEndAligner.h:31-55) */
    uint32_t location[2];      /* 0xffffffff when NotFound (the SAM writer's view) */
    uint32_t tlocation[2];     /* transcriptome location of a transcriptome record */
    int32_t  score[2];
    int32_t  mapq[2];
    uint8_t  status[2];
    uint8_t  direction[2];
    uint8_t  isTranscriptome[2];
    uint8_t  fromAlignTogether, alignedAsPair;
    uint8_t  useful;           /* passed the pre-filter */
    uint8_t  reserved[7];
} snapgpu_rna_pair_result_t;   /* 48 bytes */

typedef struct snapgpu_rna_paired_stats {
    uint64_t totalPairs, usefulPairs, singleHits, multiHits, notFound, transcriptomeRecords;
    uint64_t partialPairs, partialMatches, seedRuns;   /* FindPartialMatches scans, hits, CharacterizeSeeds runs */
    double alignMs, filterMs, seedMs, cigarMs, writeMs, wallMs;
    double prepMs;     /* clipping, ID check, pre-filter, batch views (before alignMs) */
    double countMs;    /* spacing / MAPQ adjustments and the GTF read counts (after seedMs) */
    uint64_t subBatches;   /* pipelined sub-batches (SNAPGPU_RNA_SUBBATCH pairs each; default: one): the
                              stage times above are sums over them and overlap one another in wallMs */
    double cigarGpuMs;  /* of cigarMs: the CIGAR batches (genome and transcriptome threads) */
    double spliceMs;    /* of cigarMs: insertSpliceJunctions of the transcriptome records */
    uint64_t countedPairs;  /* GTFReader::IncrementReadCount (pair form) events applied: the intragene
                               SingleHit pairs (AlignmentFilter.cpp:302-740) */
} snapgpu_rna_paired_stats_t;

/* pairedAligner: the genome aligner (snapgpu_paired_aligner_create with the paired CLI defaults);
 * transcriptomeAligner: a BaseAligner over the transcriptome index (maxHits 16000, maxK 15,
 * 8 seeds); reads0 / reads1 FASTQ batches with ids, clipped here.  samPath (or NULL) receives the
 * header and two lines per pair in input order (BAM records when it ends in ".bam"); out (or NULL)
 * one record per pair; the gtf's read counters are advanced (all of the batch's count events, or
 * none when one names an unknown transcript or gene). */
int snapgpu_rna_paired_align(snapgpu_paired_aligner_t *pairedAligner, snapgpu_aligner_t *transcriptomeAligner,
                             snapgpu_gtf_t *gtf, snapgpu_reads_t *reads0, snapgpu_reads_t *reads1,
                             const snapgpu_rna_paired_options_t *opt, const char *samPath,
                             snapgpu_rna_pair_result_t *out, snapgpu_rna_paired_stats_t *stats);
/* GTFReader::WriteReadCounts (GTFReader.cpp:1710-1772): <prefix>.{transcript,gene,junction}_{id,name}
 * .counts.txt from the gtf's read counters; snapgpu_gtf_reset_counts zeroes them. */
int snapgpu_gtf_write_counts(const snapgpu_gtf_t *gtf, const char *prefix);
int snapgpu_gtf_reset_counts(snapgpu_gtf_t *gtf);

/* MAPQ (mapq.h:32-65) as the host computes it; exported for tests. */
int snapgpu_compute_mapq(double pAll, double pBest, int score, int popularSeedsSkipped);

const char *snapgpu_last_error(void);
int snapgpu_abi_version(void);
/* This rank's host thread budget, which every host stage of the library stays within: the CPUs of
 * the affinity mask, capped by the cgroup CPU quota, divided by LOCAL_WORLD_SIZE (the ranks of the
 * node); SNAPGPU_HOST_THREADS overrides.  Read once per process.  (The reference takes `-t`,
 * ParallelTask.h:104-161.) */
int snapgpu_host_threads(void);

#ifdef __cplusplus
}
#endif
#endif /* SNAPGPU_H */

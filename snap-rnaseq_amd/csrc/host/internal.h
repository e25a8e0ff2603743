// internal.h -- host-side data structures behind the opaque handles of include/snapgpu.h.
#pragma once
#include "snapgpu.h"
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

namespace snapgpu {

// Guard bytes of 'n' before base 0 and after the last base.  The reference keeps
// N_PADDING = 100 (Genome.h:175); we keep more so that every device/host window
// [loc - 64, loc + readLen + 64) stays inside the buffer.
constexpr uint32_t kGenomeGuard = 256;
constexpr uint32_t kInvalidLocation = 0xffffffffu;   // InvalidGenomeLocation, Genome.h:29
constexpr uint32_t kUnusedSide = 0xfffffffeu;        // GenomeIndex.cpp:1511-1518
constexpr uint32_t kHashMagic = 0xb111b010u;         // HashTable.cpp:298
constexpr unsigned kQuadraticChainingDepth = 5;      // HashTable.h:115

void setError(const std::string &msg);

// threads.cpp: this rank's host thread budget -- the affinity mask capped by the cgroup CPU quota,
// divided by LOCAL_WORLD_SIZE (SNAPGPU_HOST_THREADS overrides) -- and a stage's share of it
unsigned hostThreadBudget();
unsigned hostThreads(unsigned cap);

// Host buffers the GPU copies from (read bases/qualities): page-locked when a HIP device is
// present, so the aligner's chunked H2D copies run asynchronously at PCIe speed; plain
// zeroed heap memory otherwise (build container).  *pinned says which one hostFree must undo.
// zero = false: the caller writes every byte itself (the FASTQ parser's parallel copy).
void *hostAlloc(size_t bytes, bool *pinned, bool zero = true);
void hostFree(void *p, bool pinned);

// snapgpu_reads_t::hostFlags bit 2: a view of another batch's buffers (readsView), which it does not free
constexpr uint32_t kReadsView = 4u;
snapgpu_reads_t *readsView(const snapgpu_reads_t *parent, uint64_t n, const uint64_t *offsets, const uint32_t *lengths);

struct Genome {
    std::vector<char> buf;          // guard + bases + guard (built or loaded genomes)
    const char *ext = nullptr;      // or: the same layout in a mapped shared index (snapgpu_index_attach)
    uint32_t nBases = 0;
    uint32_t chromosomePadding = 500;
    std::vector<uint32_t> pieceOffsets;
    std::vector<std::string> pieceNames;
    const char *bases() const { return (ext ? ext : buf.data()) + kGenomeGuard; }
    char *bases() { return const_cast<char *>(ext ? ext : buf.data()) + kGenomeGuard; }   // writable only when built
    // Append a contig the way ReadFASTAGenome does (FASTA.cpp:93-120): padding,
    // then the (already upper-cased, N->n) sequence.
    void reserve(uint64_t n);
    void startPiece(const std::string &name);
    void append(const char *data, size_t len);
    void appendPadding();
    void finish();                  // trailing padding + guards
};

// A read-only array that is either owned (heap, uninitialised until written) or a view into
// a mapped file (a shared index attached by another rank).
template <class T>
struct Table {
    std::unique_ptr<T[]> owned;
    const T *ptr = nullptr;
    uint64_t count = 0;
    void allocate(uint64_t n) { owned.reset(new T[n ? n : 1]); ptr = owned.get(); count = n; }
    void view(const T *p, uint64_t n) { owned.reset(); ptr = p; count = n; }
    T *mut() { return owned.get(); }
    const T *data() const { return ptr; }
    uint64_t size() const { return count; }
    bool empty() const { return count == 0; }
    const T &operator[](uint64_t i) const { return ptr[i]; }
};

struct Index {
    Genome *genome = nullptr;       // owned
    uint32_t seedLen = 20;
    uint32_t nTables = 0;
    Table<uint32_t> slots;          // 3 words per slot: key, value1, value2
    std::vector<uint64_t> tableBase;
    std::vector<uint64_t> tableSize;
    std::vector<uint64_t> tableUsed;
    Table<uint32_t> overflow;
    bool hasIupac = false;
    void *mapBase = nullptr;        // snapgpu_index_attach: the mapped shared file
    uint64_t mapLen = 0;
    ~Index();
};

// SNAPHashTable::hash (HashTable.h:60-72): MurmurHash3 fmix32.
inline uint32_t hashKey(uint32_t key) {
    key ^= key >> 16;
    key *= 0x85ebca6bu;
    key ^= key >> 13;
    key *= 0xc2b2ae35u;
    key ^= key >> 16;
    return key;
}

// Base encoding of Tables.cpp:41-48: A=0 G=1 C=2 T=3, anything else invalid (4).
inline int baseValue(char c) {
    switch (c) {
        case 'A': return 0;
        case 'G': return 1;
        case 'C': return 2;
        case 'T': return 3;
        default: return 4;
    }
}

// Host lookup with the exact probe semantics of SNAPHashTable::Lookup
// (HashTable.h:74-105).  Returns pointer to value1 or nullptr; adds probes.
const uint32_t *lookupSlot(const Index &idx, uint32_t table, uint32_t key, uint32_t *nProbes);

// One SAM line of a read without mate (SAMFormat::writeRead, SAM.cpp:1007-1155; sam.cpp).
struct SamLine {
    const char *id = nullptr;
    uint32_t idLen = 0;
    const char *bases = nullptr, *quals = nullptr;   // the unclipped read
    uint32_t fullLen = 0, front = 0, clippedLen = 0;  // unclipped length, front clip, clipped length
    int result = 0;                                   // AlignmentResult written
    uint32_t loc = kInvalidLocation;                  // writeRead's genomeLocation
    int dir = 0;
    int mapq = 0;
    int32_t ed = -1;                                  // NM (the CIGAR's edit distance), -1 = "*"
    const uint32_t *ops = nullptr;                    // BAM ops of the CIGAR, or
    uint32_t nOps = 0;
    const std::string *cigar = nullptr;               // a complete CIGAR (transcriptome records)
    const char *rg = nullptr;
    // paired records (getSAMData's hasMate branch, SAM.cpp:914-973; SimpleReadWriter::writePair,
    // ReadWriter.cpp:133-217)
    uint32_t qnameLen = 0;                            // writePair's QNAME length ("/1" "/2" dropped), 0 = idLen
    bool hasMate = false, firstInPair = false;
    uint32_t mateLoc = kInvalidLocation;              // the mate's location (invalid when NotFound)
    int mateDir = 0;
    uint32_t mateFront = 0, mateClippedLen = 0, mateFullLen = 0;
};
void samAppendLine(std::string &o, const Genome &g, const SamLine &L);
// `-so` for SAM output (SortedDataFilter::onNextBatch, SortedDataWriter.cpp:186-240, with
// SAMFormat::getSortInfo, SAM.cpp:639-685): the records of `parts` (whole lines, in write order)
// stable-sorted by their location key, concatenated
std::string samSortRecords(const Genome &g, const std::vector<std::string> &parts);
// bam.cpp: BAMFormat::writeRead of a read without mate, the BAM header, a BGZF writer
bool bamAppendRecord(std::string &o, const Genome &g, const SamLine &L, int32_t nm);
std::string bamHeader(const Genome &g, const std::string &samText);
bool bgzfWrite(FILE *f, const char *data, size_t n, bool eof);

// One pair's GTFReader::IncrementReadCount (pair form) arguments (gtf.cpp: gtfCountPairs).
struct GtfPairQuery {
    const std::string *tid0;
    uint32_t tstart0, start0, len0;
    const std::string *tid1;
    uint32_t tstart1, start1, len1;
};

// contam.cpp: ContaminationFilter::AddAlignment of every location, all or nothing (apply = false:
// only check that every location resolves)
int contaminantsAddAll(snapgpu_contaminants_t *c, const std::vector<uint32_t> &locations, bool apply = true);

}  // namespace snapgpu
// aligner.hip: snapgpu_cigar_batch over reads base[mate[i]][offsets[i] .. + lengths[i]) (no batch copy);
// two base buffers (the two ends of a pair batch, separate allocations), mate == nullptr: all base[0]
extern "C" int snapgpu_internal_cigar_view(snapgpu_aligner_t *a, const char *const base[2], const uint8_t *mate,
                                           const uint64_t *offsets,
                                           const uint32_t *lengths, uint64_t n, const uint32_t *locations,
                                           const uint8_t *directions, int useM, int32_t *editDistance, uint32_t *nOps,
                                           uint32_t *ops);
// ... the same, results left in the aligner's pinned output buffer (valid until its next CIGAR call):
// editDistance / nOps (n entries), ops (n rows of SNAPGPU_CIGAR_MAX_OPS, the first nOps of a row written)
extern "C" int snapgpu_internal_cigar_pinned(snapgpu_aligner_t *a, const char *const base[2], const uint8_t *mate,
                                             const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                                             const uint32_t *locations, const uint8_t *directions, int useM,
                                             const int32_t **editDistance, const uint32_t **nOps, const uint32_t **ops);
// aligner.hip: snapgpu_align_batch_ex with the multi-hits packed (read i: dense[off[i] .. off[i+1]))
int snapgpu_internal_align_batch_packed(snapgpu_aligner_t *a, const snapgpu_reads_t *reads,
                                        const snapgpu_search_t *search, uint32_t maxHitsToGet,
                                        snapgpu_result_t *out, int32_t *multiHitsFound, std::vector<uint64_t> &off,
                                        std::vector<snapgpu_multi_hit_t> &dense);
// ... over two batches as one (r0's reads, then r1's): one upload and one pass set
int snapgpu_internal_align_batch_packed2(snapgpu_aligner_t *a, const snapgpu_reads_t *r0, const snapgpu_reads_t *r1,
                                         uint32_t maxHitsToGet, snapgpu_result_t *out, int32_t *multiHitsFound,
                                         std::vector<uint64_t> &off, std::vector<snapgpu_multi_hit_t> &dense);
namespace snapgpu {

// xoshiro256** seeded with splitmix64: deterministic on every host.
struct Rng {
    uint64_t s[4];
    explicit Rng(uint64_t seed);
    uint64_t next();
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

}  // namespace snapgpu

struct snapgpu_genome : snapgpu::Genome {};
struct snapgpu_index : snapgpu::Index {};

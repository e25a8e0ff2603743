// rna_paired.cpp -- the RNA paired-end product path: `snap-rna paired
// <genome> <transcriptome> <gtf> r1.fq r2.fq` over a batch of pairs.
//
// PairedAlignerContext::runIterationThread (SNAPLib/PairedAligner.cpp:405-689) handles one pair
// at a time: pre-filter, two transcriptome AlignRead calls with multi-hit export (1000 hits), the
// genome ChimericPairedEndAligner, AlignmentFilter::AddAlignment for every hit,
// AlignmentFilter::Filter (AlignmentFilter.cpp:302-739) -- which for some pairs re-scans both
// reads with BaseAligner::CharacterizeSeeds (FindPartialMatches :957-1037) --, the spacing and
// MAPQ adjustments, writePair (ReadWriter.cpp:133-217) and the GTF read counts.  Here every
// stage runs over the batch: the three aligners as batched GPU calls, the filter on host
// threads, the seed census of the reads that need it as one GPU batch (charseeds_kernel), the
// count events in input order, the CIGARs as GPU batches, the SAM lines on host threads.
//
// Not restated: the contamination database (-x) and GTFReader::AnalyzeReadIntervals (the
// intra/inter-chromosomal interval report fed by UnalignedRead / *chromosomalPair): no SAM
// record or read count depends on them.
#include "internal.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace snapgpu {
struct GtfTranscript;
struct GtfGene;
const GtfTranscript *gtfTranscript(const snapgpu_gtf_t *g, const std::string &id);
const std::string &gtfTranscriptChr(const GtfTranscript *t);
const std::string &gtfTranscriptGene(const GtfTranscript *t);
uint32_t gtfGenomicPosition(const GtfTranscript *t, uint32_t pos, uint32_t span);
bool gtfSpliceCigar(const GtfTranscript *t, uint32_t pos, const std::vector<std::pair<uint32_t, char>> &tokens,
                    std::string &out);
const GtfGene *gtfGene(const snapgpu_gtf_t *g, const std::string &geneId);
bool gtfGeneCheckBoundary(const GtfGene *ge, const std::string &chr, uint32_t pos, uint32_t buffer);
int64_t gtfCountPairs(snapgpu_gtf_t *g, const std::vector<GtfPairQuery> &q);
}  // namespace snapgpu

using namespace snapgpu;

namespace {

double msSince(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int pieceAt(const Genome &g, uint32_t loc) {   // Genome::getPieceAtLocation (Genome.cpp:356-374)
    int lo = 0, hi = (int)g.pieceOffsets.size() - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (g.pieceOffsets[mid] <= loc && (mid == (int)g.pieceOffsets.size() - 1 || g.pieceOffsets[mid + 1] > loc))
            return mid;
        else if (g.pieceOffsets[mid] <= loc) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// Host worker threads of a stage: this rank's thread budget (threads.cpp: affinity, cgroup quota,
// LOCAL_WORLD_SIZE; SNAPGPU_HOST_THREADS overrides), at most 16.  The stage threads share the budget
// with the threads that drive the GPU (stage A of the next sub-batch, the CIGAR calls).  Per-thread
// arrays are sized by this, never by a constant.
static unsigned hostWorkers() {
    static const unsigned w = snapgpu::hostThreads(16);
    return w;
}

template <class F>
void parallel(uint64_t n, F &&f) {
    const unsigned nt = n < 2048 ? 1u : hostWorkers();
    if (nt == 1) { f(0u, (uint64_t)0, n); return; }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
    for (auto &x : th) x.join();
}

// The same over chunks of `chunk` items handed out by an atomic counter: for stages whose per-item
// cost is skewed (a pair's filter work grows with its alignments, up to 1000 transcriptome hits per
// read) and whose results go to per-item slots (a thread may take any chunks, in any order).
template <class F>
void parallelDyn(uint64_t n, uint64_t chunk, F &&f) {
    const unsigned nt = n < 2048 ? 1u : hostWorkers();
    if (nt == 1) { f(0u, (uint64_t)0, n); return; }
    std::atomic<uint64_t> next{0};
    auto work = [&](unsigned t) {
        for (uint64_t b; (b = next.fetch_add(chunk)) < n;) f(t, b, std::min(n, b + chunk));
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
}

const std::string kNoName;   // transcriptId / geneId of a genome alignment

// Alignment (AlignmentFilter.h:41-70).  The names point into storage that outlives the call (the
// genomes' piece names, the GTF's transcript records), so an alignment allocates nothing.
struct Alignment {
    uint32_t location = 0;
    int direction = 0;
    int score = 0, mapq = 0;
    const std::string *rname = &kNoName;
    uint32_t pos = 0, posEnd = 0, posOriginal = 0;
    bool isTranscriptome = false;
    const std::string *transcriptId = &kNoName, *geneId = &kNoName;
    const GtfGene *gene = nullptr;   // gtfGene(geneId), resolved once per transcript
};

// alignment_map's key, the string `rname + '_' + std::to_string(pos)` (AlignmentFilter.cpp:183),
// compared as that string without building it: the map's iteration order -- which the filter's
// pair lists and their std::sort inherit -- is the string order.
struct AlignKey {
    const std::string *rname;
    uint32_t pos;
    char digits[10];
    uint8_t nd;
    AlignKey(const std::string *r, uint32_t p) : rname(r), pos(p) {
        char t[10];
        int n = 0;
        do { t[n++] = (char)('0' + p % 10); p /= 10; } while (p);
        nd = (uint8_t)n;
        for (int i = 0; i < n; i++) digits[i] = t[n - 1 - i];
    }
    size_t size() const { return rname->size() + 1 + nd; }
    char at(size_t i) const {
        const size_t rn = rname->size();
        return i < rn ? (*rname)[i] : (i == rn ? '_' : digits[i - rn - 1]);
    }
};
int keyCompare(const AlignKey &a, const AlignKey &b) {
    if (a.rname == b.rname || *a.rname == *b.rname) {   // same prefix "rname_": the digit strings decide
        const int c = memcmp(a.digits, b.digits, std::min(a.nd, b.nd));
        return c ? c : (int)a.nd - (int)b.nd;
    }
    const size_t la = a.size(), lb = b.size(), l = std::min(la, lb);
    for (size_t i = 0; i < l; i++) {
        const unsigned char x = (unsigned char)a.at(i), y = (unsigned char)b.at(i);
        if (x != y) return x < y ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// alignment_map (AlignmentFilter.h: std::map<string, Alignment> keyed by rname_pos): a vector kept
// sorted by key -- the map's iteration order -- with the same find / insert / replace semantics; a
// mate holds a few entries, and clear() keeps the storage, so a pair allocates nothing
struct AlignmentMap {
    std::vector<std::pair<AlignKey, Alignment>> v;
    void clear() { v.clear(); }
    std::vector<std::pair<AlignKey, Alignment>>::iterator begin() { return v.begin(); }
    std::vector<std::pair<AlignKey, Alignment>>::iterator end() { return v.end(); }
    std::vector<std::pair<AlignKey, Alignment>>::iterator lower(const AlignKey &key) {
        return std::lower_bound(v.begin(), v.end(), key, [](const std::pair<AlignKey, Alignment> &e, const AlignKey &k) {
            return keyCompare(e.first, k) < 0;
        });
    }
};

// AlignmentPair (AlignmentFilter.cpp:63-98): score unsigned, distance int (unsigned differences)
struct AlignmentPair {
    const Alignment *a1, *a2;
    int distance = 0;
    uint32_t score = 0;
    AlignmentPair(const Alignment *x, const Alignment *y) : a1(x), a2(y) {
        score = (uint32_t)(x->score + y->score);
        if (x->direction && !y->direction) distance = (int)(x->pos - y->pos);
        else if (!x->direction && y->direction) distance = (int)(y->pos - x->pos);
    }
    bool operator<(const AlignmentPair &r) const { return score < r.score; }
};

// PairedAlignmentResult (PairedEndAligner.h:31-55) as the filter leaves it
struct PairOut {
    int status[2] = {SNAPGPU_NOT_FOUND, SNAPGPU_NOT_FOUND};
    uint32_t location[2] = {kInvalidLocation, kInvalidLocation}, tlocation[2] = {0, 0};
    int direction[2] = {0, 0}, score[2] = {0, 0}, mapq[2] = {0, 0};
    bool isTranscriptome[2] = {false, false};
    bool fromAlignTogether = false, alignedAsPair = false;
};

struct Ctx {
    const Genome *genome, *transcriptome;
    snapgpu_gtf_t *gtf;
    std::map<std::string, uint32_t> pieceByName;   // Genome::getOffsetOfPiece
    const snapgpu_rna_paired_options_t *opt;
    // per transcriptome piece: GTFReader::GetTranscript of its name (nullptr: "No transcript") and
    // GetGene of the transcript's gene (nullptr: "No gene"), looked up once per call
    std::vector<const GtfTranscript *> tByPiece;
    std::vector<const GtfGene *> gByPiece;
};

struct Err {
    std::string msg;
    void set(const std::string &m) { if (msg.empty()) msg = m; }
};

// AlignmentFilter::AddAlignment + HashAlignment (AlignmentFilter.cpp:113-214).  isMate0 picks
// map mate0 and the span of read1 (the reference's naming: read0's hits go to mate1).
void addAlignment(const Ctx &C, AlignmentMap &mate0, AlignmentMap &mate1, uint32_t location, int direction, int score,
                  int mapq, bool isT, bool isMate0, uint32_t len0, uint32_t len1, Err &err) {
    if ((uint32_t)score > C.opt->maxDist) return;   // `score > maxDist`, unsigned
    static const std::string kStar = "*";
    const std::string *rname = &kStar, *tid = &kNoName, *gid = &kNoName;
    const GtfGene *gene = nullptr;
    uint32_t pos = 0, posEnd = 0, posOriginal = 0;
    const uint32_t span = isMate0 ? len1 : len0;
    if (location != kInvalidLocation) {
        const Genome &g = isT ? *C.transcriptome : *C.genome;
        const int p = pieceAt(g, location);
        if (p < 0) { err.set("AddAlignment: location before the first piece (the reference dereferences NULL)"); return; }
        rname = &g.pieceNames[p];
        posOriginal = location - g.pieceOffsets[p] + 1;
        pos = posOriginal;
        if (!isT) {
            posEnd = pos + span - 1;
        } else {
            const GtfTranscript *t = C.tByPiece[p];
            if (!t) { err.set("No transcript " + *rname); return; }   // GTFReader::GetTranscript exits
            tid = rname;
            gid = &gtfTranscriptGene(t);
            gene = C.gByPiece[p];
            rname = &gtfTranscriptChr(t);
            posEnd = gtfGenomicPosition(t, pos + span - 1, 0);
            pos = gtfGenomicPosition(t, pos, span);
        }
    }
    if (pos == 0) return;
    AlignmentMap &m = isMate0 ? mate0 : mate1;
    const AlignKey key(rname, pos);
    auto it = m.lower(key);
    const bool isNew = it == m.end() || keyCompare(it->first, key) != 0;
    // replaced only by a lower score, or an equal transcriptome score (the element stays put)
    if (!isNew && !(score < it->second.score || (score == it->second.score && isT))) return;
    if (isNew) it = m.v.emplace(it, key, Alignment());
    Alignment &a = it->second;
    a.location = location; a.direction = direction; a.score = score; a.mapq = mapq; a.rname = rname;
    a.pos = pos; a.posEnd = posEnd; a.posOriginal = posOriginal; a.isTranscriptome = isT;
    a.transcriptId = tid; a.geneId = gid; a.gene = gene;
}

bool checkBoundary(const Alignment &a, const std::string &chr, uint32_t pos, Err &err) {
    if (!a.gene) { err.set("No gene " + *a.geneId); return false; }   // GTFReader::GetGene exits
    return gtfGeneCheckBoundary(a.gene, chr, pos, 1000);
}

// AlignmentFilter::ProcessPairs (:1061-1180)
void processPairs(const Ctx &C, PairOut &r, std::vector<AlignmentPair> &pairs, uint32_t &genomeMapq, Err &err) {
    if (pairs.size() > 1) std::sort(pairs.begin(), pairs.end());
    const AlignmentPair &p = pairs[0];
    const Alignment *a[2] = {p.a1, p.a2};
    for (int k = 0; k < 2; k++) {
        if (a[k]->isTranscriptome) {
            r.tlocation[k] = a[k]->location;
            auto po = C.pieceByName.find(*a[k]->rname);
            if (po == C.pieceByName.end()) { err.set("chromosome " + *a[k]->rname + " not in the genome"); return; }
            r.location[k] = po->second + a[k]->pos - 1;
        } else {
            r.tlocation[k] = 0;
            r.location[k] = a[k]->location;
        }
    }
    if (!a[0]->isTranscriptome && !a[1]->isTranscriptome) genomeMapq = (uint32_t)a[0]->mapq;
    for (int k = 0; k < 2; k++) {
        r.direction[k] = a[k]->direction;
        r.score[k] = a[k]->score;
        r.isTranscriptome[k] = a[k]->isTranscriptome;
    }
    const int m = (int)std::min(70u, genomeMapq);
    if (pairs.size() == 1 || pairs[1].score - pairs[0].score >= C.opt->confDiff) {
        r.status[0] = r.status[1] = SNAPGPU_SINGLE_HIT;
        r.mapq[0] = r.mapq[1] = m;
    } else {
        r.status[0] = r.status[1] = SNAPGPU_MULTIPLE_HITS;
        r.mapq[0] = r.mapq[1] = 1;
    }
}

// AlignmentFilter::CheckNoRC (:1039-1059)
void checkNoRC(PairOut &r, const std::vector<AlignmentPair> &noRc) {
    for (auto &it : noRc)
        if (*it.a1->rname == *it.a2->rname && it.score < (uint32_t)(r.score[0] + r.score[1])) {
            r.status[0] = r.status[1] = SNAPGPU_MULTIPLE_HITS;
            r.mapq[0] = r.mapq[1] = 1;
        }
}

// what AlignmentFilter::Filter (:302-739) decided for one pair before FindPartialMatches
struct FilterState {
    PairOut r;
    bool needPartial = false;    // FindPartialMatches is due (the result is SingleHit there)
    bool countPair = false;      // GTFReader::IncrementReadCount (pair form) is due
    std::string tid0, tid1;
    uint32_t tstart0 = 0, start0 = 0, len0 = 0, tstart1 = 0, start1 = 0, len1 = 0;
};

// the pair lists of one filterPair call, kept by the calling thread (cleared per pair, no allocations)
struct PairLists {
    std::vector<AlignmentPair> noRc, intragene, intra, inter;
};

void filterPair(const Ctx &C, AlignmentMap &mate0, AlignmentMap &mate1, uint32_t len0, uint32_t len1, FilterState &S,
                PairLists &L, Err &err) {
    L.noRc.clear(); L.intragene.clear(); L.intra.clear(); L.inter.clear();
    std::vector<AlignmentPair> &noRc = L.noRc, &intragene = L.intragene, &intra = L.intra, &inter = L.inter;
    uint32_t genomeMapq = 70;   // genome_mapq(maxMAPQ)
    // mate0 / mate1 empty: UnalignedRead (:742-933) only feeds the interval report (not built)
    for (auto &m0 : mate0)
        for (auto &m1 : mate1) {
            const Alignment &x = m0.second, &y = m1.second;
            if ((x.direction && y.direction) || (!x.direction && !y.direction)) { noRc.emplace_back(&y, &x); continue; }
            const bool sameChr = x.rname == y.rname || *x.rname == *y.rname;
            if (x.isTranscriptome && y.isTranscriptome) {
                if (!sameChr) inter.emplace_back(&y, &x);
                else if (checkBoundary(x, *y.rname, y.pos, err)) intragene.emplace_back(&y, &x);
                else if (checkBoundary(y, *x.rname, x.pos, err)) intragene.emplace_back(&y, &x);
                else intra.emplace_back(&y, &x);
            } else if (x.isTranscriptome) {
                if (!sameChr) inter.emplace_back(&y, &x);
                else if (checkBoundary(x, *y.rname, y.pos, err)) intragene.emplace_back(&y, &x);
                else intra.emplace_back(&y, &x);
            } else if (y.isTranscriptome) {
                if (!sameChr) inter.emplace_back(&y, &x);
                else if (checkBoundary(y, *x.rname, x.pos, err)) intragene.emplace_back(&y, &x);
                else intra.emplace_back(&y, &x);
            } else {
                intragene.emplace_back(&y, &x);
            }
        }
    PairOut &r = S.r;
    if (!intragene.empty()) {
        processPairs(C, r, intragene, genomeMapq, err);
        if (r.status[0] == SNAPGPU_SINGLE_HIT) {
            const AlignmentPair &p = intragene[0];
            S.countPair = true;
            S.tid0 = *p.a1->transcriptId; S.tstart0 = p.a1->posOriginal; S.start0 = p.a1->pos; S.len0 = len1;
            S.tid1 = *p.a2->transcriptId; S.tstart1 = p.a2->posOriginal; S.start1 = p.a2->pos; S.len1 = len0;
        }
        r.fromAlignTogether = false;
        r.alignedAsPair = true;
        return;
    }
    if (!intra.empty()) {
        processPairs(C, r, intra, genomeMapq, err);
        if (r.status[0] == SNAPGPU_SINGLE_HIT) checkNoRC(r, noRc);
        if ((uint32_t)intra[0].distance <= C.opt->maxSpacing) return;   // flags left as the chimeric aligner set them
        S.needPartial = r.status[0] == SNAPGPU_SINGLE_HIT;
        r.fromAlignTogether = false;
        r.alignedAsPair = false;
        return;
    }
    if (!inter.empty()) {
        processPairs(C, r, inter, genomeMapq, err);
        if (r.status[0] == SNAPGPU_SINGLE_HIT) checkNoRC(r, noRc);
        S.needPartial = r.status[0] == SNAPGPU_SINGLE_HIT;
        r.fromAlignTogether = false;
        r.alignedAsPair = false;
        return;
    }
    if (!noRc.empty()) {
        processPairs(C, r, noRc, genomeMapq, err);
        S.needPartial = r.status[0] == SNAPGPU_SINGLE_HIT;
        r.fromAlignTogether = false;
        r.alignedAsPair = false;
        return;
    }
    for (int k = 0; k < 2; k++) {
        r.tlocation[k] = 0; r.status[k] = SNAPGPU_NOT_FOUND; r.location[k] = 0; r.direction[k] = 0;
        r.score[k] = 0; r.mapq[k] = 0; r.isTranscriptome[k] = false;
    }
    r.fromAlignTogether = false;
    r.alignedAsPair = false;
}

// FindPartialMatches (:957-1037): any pair of seed-run starts of the two reads on one
// chromosome closer than maxSpacing (the reference's double loop, as a sorted sweep)
bool partialMatch(const Ctx &C, const snapgpu_seed_runs_t *R, uint64_t i0, uint64_t i1, uint32_t len0, uint32_t len1,
                  Err &err) {
    std::vector<std::pair<int, int>> p[2];   // (piece, 1-based position)
    const uint64_t ri[2] = {i0, i1};
    const uint32_t lens[2] = {len0, len1};
    for (int k = 0; k < 2; k++)
        for (uint64_t j = R->start[ri[k]]; j < R->start[ri[k] + 1]; j++) {
            const snapgpu_seed_run_t &run = R->runs[j];
            const uint32_t loc = run.direction ? run.location + (lens[k] - run.maxOffset) : run.location + run.minOffset;
            const int pc = pieceAt(*C.genome, loc);
            if (pc < 0) { err.set("FindPartialMatches: location before the first piece (the reference dereferences NULL)"); return false; }
            p[k].push_back({pc, (int)(loc - C.genome->pieceOffsets[pc] + 1)});
        }
    std::sort(p[1].begin(), p[1].end());
    for (auto &a : p[0]) {
        // closest positions of the other read on the same piece
        auto it = std::lower_bound(p[1].begin(), p[1].end(), a);
        for (int d = 0; d < 2; d++) {
            auto b = d == 0 ? it : (it == p[1].begin() ? p[1].end() : it - 1);
            if (b == p[1].end() || b->first != a.first) continue;
            if ((uint32_t)std::abs(b->second - a.second) < C.opt->maxSpacing) return true;
        }
    }
    return false;
}

bool idsMatch(const char *a, uint32_t la, const char *b, uint32_t lb) {   // readIdsMatch (SAM.cpp:53-68)
    if (la != lb) return false;
    for (uint32_t i = 0; i < la; i++) {
        if (a[i] != b[i]) return false;
        if (a[i] == ' ' || a[i] == '/') return true;
    }
    return true;
}


// One snapgpu_rna_paired_align call: what its sub-batches share.
struct RnaRun {
    snapgpu_paired_aligner_t *pa;
    snapgpu_aligner_t *ta, *ga;
    const snapgpu_index_t *gi, *ti;
    snapgpu_gtf_t *gtf;
    snapgpu_reads_t *R[2];
    const snapgpu_rna_paired_options_t *opt;
    const std::vector<uint8_t> *useful;
    std::mutex *mT, *mG;   // the transcriptome / genome aligner's align calls
    // their CIGAR / seed-census calls: the aligners' side stream and buffers (aligner.hip), so stage
    // B of one sub-batch runs them while stage A of the next holds mT / mG
    std::mutex *mTs, *mGs;
    const Ctx *C;
    bool bam;
};

// Pairs [a, b) of the batch through the path; stage A fills the aligner outputs, stage B the rest.
struct RnaSub {
    uint64_t a = 0, b = 0;
    std::vector<uint64_t> ui;                 // the useful pairs (batch indices)
    snapgpu_reads_t *U[2] = {nullptr, nullptr};
    std::vector<uint64_t> uo[2];
    std::vector<uint32_t> ul[2];
    // the transcriptome aligner's records of both ends, end k of useful pair j at k * nu + j, and
    // its hits: th[thOff[k * nu + j] .. thOff[k * nu + j + 1])
    std::vector<snapgpu_result_t> tr;
    std::vector<int32_t> tf;
    std::vector<uint64_t> thOff;
    std::vector<snapgpu_multi_hit_t> th;
    std::vector<snapgpu_pair_result_t> gr;
    std::vector<FilterState> fs;              // per useful pair
    std::vector<GtfPairQuery> cq;             // count events (pointing into fs), input order
    std::vector<uint32_t> contamLocs;         // -ct: both ends of the pairs the contamination aligner placed
    std::vector<PairOut> po;                  // per pair of [a, b)
    std::vector<std::string> parts;           // the SAM lines / BAM records of [a, b), in order
    uint64_t single = 0, multi = 0, notFound = 0, partialPairs = 0, partialMatches = 0, seedRuns = 0;
    uint64_t transcriptomeRecords = 0;
    double alignMs = 0, filterMs = 0, seedMs = 0, countMs = 0, cigarMs = 0, writeMs = 0, cigarGpuMs = 0, spliceMs = 0;
    int rc = SNAPGPU_OK;
    std::string err;
    RnaSub() = default;
    RnaSub(const RnaSub &) = delete;
    ~RnaSub() { snapgpu_reads_free(U[0]); snapgpu_reads_free(U[1]); }
    void fail(int code, const std::string &m) { if (rc == SNAPGPU_OK) { rc = code; err = m; } }
};

// Stage A: the useful pairs' batch views, the transcriptome AlignRead of both ends with 1000
// multi-hits (PairedAligner.cpp:601-605) and, on a thread of its own, the genome
// ChimericPairedEndAligner (:625) -- the two aligners have their own streams and device buffers.
void rnaStageA(const RnaRun &Rr, RnaSub &X) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = X.a; i < X.b; i++) if ((*Rr.useful)[i]) X.ui.push_back(i);
    const uint64_t nu = X.ui.size();
    for (int k = 0; k < 2; k++) {
        X.uo[k].resize(nu + 1); X.ul[k].resize(nu + 1);
        for (uint64_t j = 0; j < nu; j++) { X.uo[k][j] = Rr.R[k]->offsets[X.ui[j]]; X.ul[k][j] = Rr.R[k]->lengths[X.ui[j]]; }
        X.U[k] = readsView(Rr.R[k], nu, X.uo[k].data(), X.ul[k].data());   // no copy of the reads
        if (!X.U[k]) { X.fail(SNAPGPU_ENOMEM, "rna_paired_align: out of memory"); return; }
    }
    X.gr.resize(nu + 1);
    if (nu) {
        int grc = SNAPGPU_OK;
        std::string gerr;
        auto genomePairs = [&] {
            std::lock_guard<std::mutex> lk(*Rr.mG);
            grc = snapgpu_paired_align_batch(Rr.pa, X.U[0], X.U[1], X.gr.data());
            if (grc) gerr = snapgpu_last_error();
        };
        const bool overlap = Rr.ta != Rr.ga;
        std::thread gt;
        if (overlap) gt = std::thread(genomePairs);
        int rc = SNAPGPU_OK;
        std::string terr;
        {
            std::lock_guard<std::mutex> lk(*Rr.mT);
            // both ends in one call: one persistent-kernel tail instead of two
            X.tr.resize(2 * nu); X.tf.resize(2 * nu);
            rc = snapgpu_internal_align_batch_packed2(Rr.ta, X.U[0], X.U[1], Rr.opt->maxHitsToGet, X.tr.data(), X.tf.data(),
                                                      X.thOff, X.th);
            if (rc) terr = snapgpu_last_error();
        }
        if (overlap) gt.join();
        else if (rc == SNAPGPU_OK) genomePairs();
        if (rc) { X.fail(rc, terr); return; }
        if (grc) { X.fail(grc, gerr); return; }
    }
    X.alignMs = msSince(t0);
}

// Stage B: AlignmentFilter (AddAlignment + Filter, AlignmentFilter.cpp:113-739) on host threads,
// FindPartialMatches' seed census as one GPU batch, the spacing / MAPQ adjustments and the count
// events (PairedAligner.cpp:648-663), the CIGARs of both ends as GPU batches (genome; transcriptome
// + insertSpliceJunctions) and the records of writePair (ReadWriter.cpp:133-217).  lastNm: the BAM
// NM carry-over from the previous sub-batch (the reference's writeRead leaves an unmapped record
// with the previous record's editDistance).
void rnaStageB(const RnaRun &Rr, RnaSub &X, int32_t &lastNm) {
    const Ctx &C = *Rr.C;
    const snapgpu_rna_paired_options_t *opt = Rr.opt;
    snapgpu_reads_t *const *R = Rr.R;
    const uint64_t nu = X.ui.size(), nb = X.b - X.a;
    auto t0 = std::chrono::steady_clock::now();
    X.fs.assign(nu + 1, FilterState());
    std::vector<Err> errs(hostWorkers());
    parallelDyn(nu, 512, [&](unsigned t, uint64_t b, uint64_t e) {
        AlignmentMap mate0, mate1;
        PairLists lists;
        for (uint64_t j = b; j < e && errs[t].msg.empty(); j++) {
            mate0.clear(); mate1.clear();
            const uint32_t len0 = X.ul[0][j], len1 = X.ul[1][j];
            for (int k = 0; k < 2 && !X.thOff.empty(); k++)   // (no hits asked for: none recorded)
                for (uint64_t h = X.thOff[k * nu + j]; h < X.thOff[k * nu + j + 1]; h++) {
                    const snapgpu_multi_hit_t &m = X.th[h];
                    addAlignment(C, mate0, mate1, m.location, m.direction, m.score, 0, true, k == 1, len0, len1, errs[t]);
                }
            const snapgpu_pair_result_t &g = X.gr[j];
            addAlignment(C, mate0, mate1, g.location[0], g.direction[0], g.score[0], g.mapq[0], false, false, len0, len1, errs[t]);
            addAlignment(C, mate0, mate1, g.location[1], g.direction[1], g.score[1], g.mapq[1], false, true, len0, len1, errs[t]);
            FilterState &S = X.fs[j];
            S.r.fromAlignTogether = g.fromAlignTogether;
            S.r.alignedAsPair = g.alignedAsPair;
            filterPair(C, mate0, mate1, len0, len1, S, lists, errs[t]);
        }
    });
    for (auto &e : errs) if (!e.msg.empty()) { X.fail(SNAPGPU_EFORMAT, "rna_paired_align: " + e.msg); return; }
    X.filterMs = msSince(t0);
    // CIGARs on the GPU (writeRead, SAM.cpp:1040-1066): genome records at the location, the
    // transcriptome records on the transcriptome at tlocation.  Only the records with a location
    // go to the GPU, as compact batches (a read without one has no CIGAR: edit distance -1, no
    // ops).  Which records have a location, where and on which index is settled by the filter:
    // FindPartialMatches only turns a pair with both ends SingleHit into MultipleHits, and the
    // spacing adjustment only takes locations away (a row computed for such a record is never
    // read: its line has no location).  So the CIGAR batches are launched here, on a host thread
    // of their own, and run on the GPU while this thread does the seed census, the contamination
    // pass and the count events; the genome (ga) and transcriptome (ta) batches overlap each other
    // when the aligners are distinct.
    auto tc0 = std::chrono::steady_clock::now();
    // Both ends of the sub-batch in one set per aligner, one GPU call each: a row is addressed by
    // its end's buffer and its offset there (no copy of the batch, no pointer arithmetic across the
    // two allocations).
    const char *const cbase[2] = {R[0]->bases, R[1]->bases};
    struct CigarSet {
        std::vector<int64_t> slot[2];   // end k, record -> row in ed/nOps/ops, -1: no location
        std::vector<uint64_t> off;      // in the row's end's buffer
        std::vector<uint8_t> mate;      // the row's end
        std::vector<uint32_t> len, loc, nOps;
        std::unique_ptr<uint32_t[]> ops;   // [rows][SNAPGPU_CIGAR_MAX_OPS], every row written by the download
        std::vector<uint8_t> dir;
        std::vector<int32_t> ed;
        int32_t edOf(int k, uint64_t i) const { return slot[k][i] >= 0 ? ed[slot[k][i]] : -1; }
        uint32_t nOpsOf(int k, uint64_t i) const { return slot[k][i] >= 0 ? nOps[slot[k][i]] : 0u; }
        const uint32_t *opsOf(int k, uint64_t i) const {
            static const uint32_t kNone[1] = {0};
            return slot[k][i] >= 0 ? ops.get() + slot[k][i] * SNAPGPU_CIGAR_MAX_OPS : kNone;
        }
        void add(int k, uint64_t i, uint64_t o, uint32_t ln, uint32_t l, uint8_t d) {
            slot[k][i] = (int64_t)loc.size();
            off.push_back(o);
            mate.push_back((uint8_t)k);
            len.push_back(ln);
            loc.push_back(l);
            dir.push_back(d);
        }
        uint64_t rows() const { return loc.size(); }
        int run(snapgpu_aligner_t *a, const char *const base[2], int useM, std::mutex &m) {
            const uint64_t cnt = loc.size();
            ed.assign(cnt + 1, -1);
            nOps.assign(cnt + 1, 0);
            ops.reset(new uint32_t[(cnt + 1) * SNAPGPU_CIGAR_MAX_OPS]);
            if (!cnt) return SNAPGPU_OK;
            std::lock_guard<std::mutex> lk(m);
            return snapgpu_internal_cigar_view(a, base, mate.data(), off.data(), len.data(), cnt, loc.data(), dir.data(), useM, ed.data(),
                                               nOps.data(), ops.get());
        }
    };
    CigarSet gc, tc;
    for (int k = 0; k < 2; k++) {
        gc.slot[k].assign(nb, -1);
        tc.slot[k].assign(nb, -1);
        for (uint64_t j = 0; j < nu; j++) {
            const PairOut &r = X.fs[j].r;
            const uint64_t i = X.ui[j], q = i - X.a;
            const uint32_t loc = r.status[k] != SNAPGPU_NOT_FOUND ? r.location[k] : kInvalidLocation;
            if (loc == kInvalidLocation) continue;
            const uint64_t o = R[k]->offsets[i];
            if (r.isTranscriptome[k]) tc.add(k, q, o, R[k]->lengths[i], r.tlocation[k], (uint8_t)r.direction[k]);
            else gc.add(k, q, o, R[k]->lengths[i], loc, (uint8_t)r.direction[k]);
        }
    }
    double cigarBuildMs = msSince(tc0);
    int grc = SNAPGPU_OK, trc = SNAPGPU_OK;
    std::string gerr, terr;
    // the seed census below is on this thread's critical path and shares the genome aligner's side
    // stream with the genome CIGARs: those wait until the census has been issued and returned
    std::promise<void> censusDone;
    std::shared_future<void> censusDoneF = censusDone.get_future().share();
    struct Joiner {
        std::promise<void> *census;
        std::thread t;
        bool released = false;
        void release() { if (!released) { released = true; census->set_value(); } }
        ~Joiner() { release(); if (t.joinable()) t.join(); }   // every return below waits for the GPU calls
    } cig{&censusDone};
    cig.t = std::thread([&] {
        const auto tg0 = std::chrono::steady_clock::now();
        // one aligner's stream, events and upload state serve one host thread at a time (mTs is mGs
        // when the transcriptome and genome aligners are one)
        if (Rr.ta == Rr.ga) censusDoneF.wait();
        trc = tc.run(Rr.ta, cbase, (int)opt->useM, *Rr.mTs);
        if (trc) terr = snapgpu_last_error();
        censusDoneF.wait();
        if (trc == SNAPGPU_OK) {
            grc = gc.run(Rr.ga, cbase, (int)opt->useM, *Rr.mGs);
            if (grc) gerr = snapgpu_last_error();
        }
        X.cigarGpuMs = msSince(tg0);
    });
    // FindPartialMatches: CharacterizeSeeds of both reads of the pairs that need it, one GPU batch
    t0 = std::chrono::steady_clock::now();
    std::vector<uint64_t> need;
    for (uint64_t j = 0; j < nu; j++) if (X.fs[j].needPartial) need.push_back(j);
    X.partialPairs = need.size();
    if (!need.empty()) {
        // both reads in one batch: read0 of need[i] at 2i, read1 at 2i + 1
        std::vector<uint64_t> po(2 * need.size() + 1);
        std::vector<uint32_t> pl(2 * need.size() + 1);
        std::string bb, qq;
        for (size_t i = 0; i < need.size(); i++)
            for (int k = 0; k < 2; k++) {
                const uint64_t o = X.uo[k][need[i]];
                po[2 * i + k] = bb.size();
                pl[2 * i + k] = X.ul[k][need[i]];
                bb.append(R[k]->bases + o, X.ul[k][need[i]]);
                qq.append(R[k]->quals + o, X.ul[k][need[i]]);
            }
        snapgpu_reads_t *both = snapgpu_reads_from_arrays(2 * need.size(), bb.data(), qq.data(), po.data(), pl.data());
        if (!both) { X.fail(SNAPGPU_ENOMEM, "rna_paired_align: out of memory"); return; }
        snapgpu_charseeds_params_t cp;
        snapgpu_charseeds_params_default(&cp);   // the partial aligner: maxHits 300, 12 seeds (:518-527)
        cp.maxK = opt->maxDist;
        snapgpu_seed_runs_t *runs;
        {
            std::lock_guard<std::mutex> lk(*Rr.mGs);
            runs = snapgpu_characterize_seeds(Rr.ga, both, nullptr, 0, &cp);
            if (!runs) X.fail(SNAPGPU_EDEVICE, snapgpu_last_error());
        }
        snapgpu_reads_free(both);
        cig.release();
        if (!runs) return;
        std::unique_ptr<snapgpu_seed_runs_t, void (*)(snapgpu_seed_runs_t *)> hold(runs, snapgpu_seed_runs_free);
        for (uint64_t i = 0; i < 2 * need.size(); i++)
            if (runs->flags[i] & SNAPGPU_FLAG_READ_TOO_LONG) {
                X.fail(SNAPGPU_EINVAL, "rna_paired_align: read longer than maxReadSize (the reference exits, BaseAligner.cpp:272-275)");
                return;
            }
        X.seedRuns = runs->nRuns;
        std::vector<uint8_t> hit(need.size(), 0);
        parallelDyn(need.size(), 256, [&](unsigned t, uint64_t b, uint64_t e) {
            for (uint64_t i = b; i < e; i++)
                hit[i] = partialMatch(C, runs, 2 * i, 2 * i + 1, X.ul[0][need[i]], X.ul[1][need[i]], errs[t]);
        });
        for (auto &e : errs) if (!e.msg.empty()) { X.fail(SNAPGPU_EFORMAT, "rna_paired_align: " + e.msg); return; }
        for (size_t i = 0; i < need.size(); i++)
            if (hit[i]) {
                PairOut &r = X.fs[need[i]].r;
                r.status[0] = r.status[1] = SNAPGPU_MULTIPLE_HITS;
                r.mapq[0] = r.mapq[1] = 1;
                X.partialMatches++;
            }
    }
    cig.release();   // (no census batch)
    X.seedMs = msSince(t0);
    t0 = std::chrono::steady_clock::now();
    // -ct (PairedAligner.cpp:632-645): pairs still NotFound on both ends through the contamination
    // paired aligner, one GPU batch; a pair it aligns on both ends adds both ends' contigs
    if (opt->contaminationAligner && opt->contaminants) {
        std::vector<uint64_t> co[2];
        std::vector<uint32_t> cl[2];
        for (uint64_t j = 0; j < nu; j++) {
            const PairOut &r = X.fs[j].r;
            if (r.status[0] != SNAPGPU_NOT_FOUND || r.status[1] != SNAPGPU_NOT_FOUND) continue;
            for (int k = 0; k < 2; k++) { co[k].push_back(X.uo[k][j]); cl[k].push_back(X.ul[k][j]); }
        }
        if (!co[0].empty()) {
            snapgpu_reads_t *cv[2];
            for (int k = 0; k < 2; k++) cv[k] = readsView(R[k], co[k].size(), co[k].data(), cl[k].data());
            std::vector<snapgpu_pair_result_t> cr(co[0].size());
            int rc = cv[0] && cv[1] ? snapgpu_paired_align_batch(opt->contaminationAligner, cv[0], cv[1], cr.data()) : SNAPGPU_ENOMEM;
            if (rc && rc != SNAPGPU_ENOMEM) X.fail(rc, snapgpu_last_error());
            else if (rc) X.fail(rc, "rna_paired_align: out of memory");
            for (auto *v : cv) snapgpu_reads_free(v);
            if (X.rc != SNAPGPU_OK) return;
            for (auto &r : cr)   // added with the GTF counts at the end of the call, all or nothing
                if (r.status[0] != SNAPGPU_NOT_FOUND && r.status[1] != SNAPGPU_NOT_FOUND)
                    for (int k = 0; k < 2; k++) X.contamLocs.push_back(r.location[k]);
        }
    }
    // spacing and MAPQ adjustments (PairedAligner.cpp:648-663); the count events in input order
    // (applied for the whole batch at the end: gtfCountPairs)
    for (uint64_t j = 0; j < nu; j++) {
        PairOut &r = X.fs[j].r;
        if (opt->forceSpacing && (r.status[0] == SNAPGPU_SINGLE_HIT) != (r.status[1] == SNAPGPU_SINGLE_HIT)) {
            r.status[0] = r.status[1] = SNAPGPU_NOT_FOUND;
            r.location[0] = r.location[1] = kInvalidLocation;
        }
        if (r.score[0] + r.score[1] >= 5)
            for (int k = 0; k < 2; k++) if (r.mapq[k] < 50) r.mapq[k] /= 2;
        const FilterState &S = X.fs[j];
        if (S.countPair) X.cq.push_back(GtfPairQuery{&S.tid0, S.tstart0, S.start0, S.len0, &S.tid1, S.tstart1, S.start1, S.len1});
    }
    // the pairs' records, in input order; filtered pairs: NotFound, InvalidGenomeLocation
    X.po.assign(nb, PairOut());
    for (uint64_t j = 0; j < nu; j++) X.po[X.ui[j] - X.a] = X.fs[j].r;
    X.countMs = msSince(t0);
    // the final records' index: transcriptome records are the ones with a location on it
    t0 = std::chrono::steady_clock::now();
    std::vector<uint8_t> isT[2];
    for (int k = 0; k < 2; k++) {
        isT[k].assign(nb, 0);
        for (uint64_t q = 0; q < nb; q++) {
            const PairOut &r = X.po[q];
            const uint32_t loc = r.status[k] != SNAPGPU_NOT_FOUND ? r.location[k] : kInvalidLocation;
            isT[k][q] = loc != kInvalidLocation && r.isTranscriptome[k];
            X.transcriptomeRecords += isT[k][q];
        }
    }
    cig.t.join();
    if (trc) { X.fail(trc, terr); return; }
    if (grc) { X.fail(grc, gerr); return; }
    // transcriptome records: computeCigarString's tokens through insertSpliceJunctions
    const auto ts0 = std::chrono::steady_clock::now();
    const Genome &tg = *Rr.ti->genome;
    std::vector<std::string> splice[2];
    for (int k = 0; k < 2; k++) {
        splice[k].assign(nb, std::string());
        parallelDyn(nb, 1024, [&](unsigned, uint64_t b, uint64_t e) {
            std::vector<std::pair<uint32_t, char>> tk;
            static const char kOp[] = "MIDNSHP=X";
            for (uint64_t q = b; q < e; q++) {
                if (!isT[k][q]) continue;
                tk.clear();
                const PairOut &r = X.po[q];
                const uint64_t i = X.a + q;
                if (tc.edOf(k, q) >= 0) {
                    const uint32_t full = R[k]->unclippedLength[i], front = R[k]->frontClipped[i];
                    const uint32_t back = full - R[k]->lengths[i] - front;
                    const bool rcd = r.direction[k] == SNAPGPU_RC;
                    const uint32_t before = rcd ? back : front, after = rcd ? front : back;
                    if (before) tk.push_back({before, 'S'});
                    const uint32_t *tops = tc.opsOf(k, q);
                    for (uint32_t z = 0; z < tc.nOpsOf(k, q); z++) {
                        const uint32_t op = tops[z];
                        tk.push_back({op >> 4, kOp[op & 15]});
                    }
                    if (after) tk.push_back({after, 'S'});
                }
                const int p = pieceAt(tg, r.tlocation[k]);
                const GtfTranscript *t = p >= 0 ? C.tByPiece[p] : nullptr;
                if (t) gtfSpliceCigar(t, r.tlocation[k] - tg.pieceOffsets[p] + 1, tk, splice[k][q]);
            }
        });
    }
    X.spliceMs = msSince(ts0);
    X.cigarMs = cigarBuildMs + msSince(t0);
    // writePair (ReadWriter.cpp:133-217): the end at the lower location first
    t0 = std::chrono::steady_clock::now();
    const unsigned ntd = nb < 2048 ? 1u : hostWorkers();
    // the records in chunks of WCH pairs handed out dynamically, one part per chunk: the parts
    // concatenate in chunk order, i.e. input order, whichever thread wrote them
    constexpr uint64_t WCH = 1024;
    std::vector<std::string> parts((nb + WCH - 1) / WCH);
    std::vector<uint64_t> cnt(16 * ntd, 0);   // thread t's three counters at 16 t: a cache line of their own
    // BAM: NM is set only for a record with a location; the others repeat the previous record's
    // value, so a serial pass in write order fixes each record's NM
    std::vector<int32_t> bamNm;
    std::vector<uint8_t> bamBad(ntd, 0);
    if (Rr.bam) {
        bamNm.resize(2 * nb);
        for (uint64_t q = 0; q < nb; q++) {
            const PairOut &r = X.po[q];
            uint32_t locs[2];
            for (int k = 0; k < 2; k++) locs[k] = r.status[k] != SNAPGPU_NOT_FOUND ? r.location[k] : kInvalidLocation;
            const int first = locs[0] > locs[1];
            for (int w = 0; w < 2; w++) {
                const int k = w == 0 ? first : 1 - first;
                if (locs[k] != kInvalidLocation) lastNm = isT[k][q] ? tc.edOf(k, q) : gc.edOf(k, q);
                bamNm[2 * q + w] = lastNm;
            }
        }
    }
    const Genome &gg = *Rr.gi->genome;
    parallelDyn(nb, WCH, [&](unsigned t, uint64_t b, uint64_t e) {
        // a local string swapped in at the end (the parts' headers share cache lines: appending
        // through them bounced those lines between the writer threads)
        std::string o;
        o.reserve((e - b) * 640);
        for (uint64_t q = b; q < e; q++) {
            const PairOut &r = X.po[q];
            const uint64_t i = X.a + q;
            uint32_t idLen[2] = {R[0]->idLengths[i], R[1]->idLengths[i]};
            const char *id[2] = {R[0]->ids + R[0]->idOffsets[i], R[1]->ids + R[1]->idOffsets[i]};
            if (idLen[0] == idLen[1] && idLen[0] > 2 && id[0][idLen[0] - 2] == '/' && id[1][idLen[0] - 2] == '/') {
                const char c0 = id[0][idLen[0] - 1], c1 = id[1][idLen[1] - 1];
                if ((c0 == '1' || c0 == '2') && (c0 == '1' || c1 == '2') && c0 != c1) { idLen[0] -= 2; idLen[1] -= 2; }
            }
            uint32_t locs[2];
            for (int k = 0; k < 2; k++) locs[k] = r.status[k] != SNAPGPU_NOT_FOUND ? r.location[k] : kInvalidLocation;
            const int first = locs[0] > locs[1], second = 1 - first;
            for (int w = 0; w < 2; w++) {
                const int k = w == 0 ? first : second, m = 1 - k;
                SamLine L;
                L.id = id[k];
                L.idLen = R[k]->idLengths[i];
                L.qnameLen = idLen[k];
                L.front = R[k]->frontClipped[i];
                L.clippedLen = R[k]->lengths[i];
                L.fullLen = R[k]->unclippedLength[i];
                L.bases = R[k]->bases + R[k]->offsets[i] - L.front;
                L.quals = R[k]->quals + R[k]->offsets[i] - L.front;
                L.rg = opt->readGroup;
                L.result = r.status[k];
                L.loc = locs[k];
                L.dir = r.direction[k];
                L.mapq = r.mapq[k];
                if (isT[k][q]) {
                    L.cigar = &splice[k][q];
                    L.ed = tc.edOf(k, q);
                } else {
                    L.ed = gc.edOf(k, q);
                    L.ops = gc.opsOf(k, q);
                    L.nOps = gc.nOpsOf(k, q);
                }
                L.hasMate = true;
                L.firstInPair = w == 0;
                L.mateLoc = locs[m];
                L.mateDir = r.direction[m];
                L.mateFront = R[m]->frontClipped[i];
                L.mateClippedLen = R[m]->lengths[i];
                L.mateFullLen = R[m]->unclippedLength[i];
                if (!Rr.bam) samAppendLine(o, gg, L);
                else if (!bamAppendRecord(o, gg, L, bamNm[2 * q + w])) bamBad[t] = 1;
                cnt[16 * t + (r.status[k] == SNAPGPU_SINGLE_HIT ? 0 : r.status[k] == SNAPGPU_MULTIPLE_HITS ? 1 : 2)]++;
            }
        }
        parts[b / WCH].swap(o);
    });
    for (unsigned t = 0; t < ntd; t++)
        if (bamBad[t]) {
            X.fail(SNAPGPU_EINVAL, "rna_paired_align: BAM record not written (QNAME longer than 254 characters, Bam.cpp:723-726)");
            return;
        }
    for (unsigned t = 0; t < ntd; t++) { X.single += cnt[16 * t]; X.multi += cnt[16 * t + 1]; X.notFound += cnt[16 * t + 2]; }
    X.parts.swap(parts);
    X.writeMs = msSince(t0);
}

}  // namespace

extern "C" {

void snapgpu_rna_paired_options_default(snapgpu_rna_paired_options_t *o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->clipping = 3;              // AlignerOptions.cpp:48
    o->confDiff = 2;
    o->maxDist = 15;              // AlignerOptions.cpp:73-77 (paired)
    o->minSpacing = 50;           // PairedAligner.cpp:57-58
    o->maxSpacing = 1000;
    o->minPercentAbovePhred = 90.0f;
    o->minPhred = 20;
    o->phredOffset = 33;
    o->maxHitsToGet = 1000;       // PairedAligner.cpp:584
    o->readGroup = "FASTQ";
    o->commandLine = "";
    o->version = "";
}

int snapgpu_rna_paired_align(snapgpu_paired_aligner_t *pa, snapgpu_aligner_t *ta, snapgpu_gtf_t *gtf,
                             snapgpu_reads_t *reads0, snapgpu_reads_t *reads1, const snapgpu_rna_paired_options_t *opt,
                             const char *samPath, snapgpu_rna_pair_result_t *out, snapgpu_rna_paired_stats_t *stats) {
    const auto w0 = std::chrono::steady_clock::now();
    if (!pa || !ta || !gtf || !reads0 || !reads1 || !opt) { setError("rna_paired_align: null argument"); return SNAPGPU_EINVAL; }
    if (reads0->n != reads1->n) { setError("rna_paired_align: the two read batches differ in length"); return SNAPGPU_EINVAL; }
    if (opt->sortOutput && samPath && strlen(samPath) >= 4 && strcmp(samPath + strlen(samPath) - 4, ".bam") == 0) {
        setError("rna_paired_align: sorted output is built for SAM only");   // sorted BAM + BAMIndexSupplier's .bai
        return SNAPGPU_EUNSUPPORTED;
    }
    if (!reads0->ids || !reads1->ids) { setError("rna_paired_align: the reads carry no ids (use snapgpu_reads_from_fastq)"); return SNAPGPU_EINVAL; }
    snapgpu_aligner_t *ga = snapgpu_paired_aligner_single(pa);   // the genome index upload (BaseAligner)
    const snapgpu_index_t *gi = snapgpu_aligner_index(ga), *ti = snapgpu_aligner_index(ta);
    if (!gi || !ti) { setError("rna_paired_align: aligner without index"); return SNAPGPU_EINVAL; }
    snapgpu_rna_paired_stats_t st{};
    const uint64_t n = reads0->n;
    st.totalPairs = n;
    snapgpu_reads_t *R[2] = {reads0, reads1};
    for (int k = 0; k < 2; k++) {
        const int rc = snapgpu_reads_clip(R[k], opt->clipping, nullptr, nullptr);   // FASTQReader (FASTQ.cpp:250)
        if (rc) return rc;
    }
    if (!opt->ignoreMismatchedIDs) {   // Read::checkIdMatch (Read.cpp:37-49): the reference exits
        std::vector<uint64_t> bad(hostWorkers(), n);   // first mismatching pair of each thread's range
        parallel(n, [&](unsigned t, uint64_t b, uint64_t e) {
            for (uint64_t i = b; i < e; i++)
                if (!idsMatch(reads0->ids + reads0->idOffsets[i], reads0->idLengths[i],
                              reads1->ids + reads1->idOffsets[i], reads1->idLengths[i])) { bad[t] = i; break; }
        });
        const uint64_t i = *std::min_element(bad.begin(), bad.end());
        if (i < n) {
            setError("rna_paired_align: unmatched read IDs at pair " + std::to_string(i) + " (ignoreMismatchedIDs)");
            return SNAPGPU_EINVAL;
        }
    }
    // pre-filter (PairedAligner.cpp:555-575): length / Ns per read, quality of read0 (sic, :564)
    std::vector<uint8_t> useful(n, 0);
    parallel(n, [&](unsigned, uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            bool u[2], q[2];
            for (int k = 0; k < 2; k++) {
                const char *d = R[k]->bases + R[k]->offsets[i], *qq = R[k]->quals + R[k]->offsets[i];
                const uint32_t len = R[k]->lengths[i];
                unsigned ns = 0, good = 0;
                for (uint32_t j = 0; j < len; j++) {
                    ns += d[j] == 'N' || d[j] == 'n';
                    good += (unsigned)(int)qq[j] - opt->phredOffset >= opt->minPhred;
                }
                u[k] = len >= 50 && (int)ns <= (int)opt->maxDist;
                q[k] = ((float)good / (float)len) * 100.f >= opt->minPercentAbovePhred;
            }
            useful[i] = !((!u[0] && !u[1]) || !q[0]);
        }
    });
    for (uint64_t i = 0; i < n; i++) st.usefulPairs += useful[i];
    st.prepMs = msSince(w0);
    Ctx C{gi->genome, ti->genome, gtf, {}, opt};
    for (size_t p = 0; p < gi->genome->pieceNames.size(); p++) C.pieceByName.insert({gi->genome->pieceNames[p], gi->genome->pieceOffsets[p]});
    for (const std::string &name : ti->genome->pieceNames) {
        const GtfTranscript *t = gtfTranscript(gtf, name);
        C.tByPiece.push_back(t);
        C.gByPiece.push_back(t ? gtfGene(gtf, gtfTranscriptGene(t)) : nullptr);
    }
    const size_t spl = samPath ? strlen(samPath) : 0;
    // BAM when the path ends in ".bam" (BAMFormat::writeRead for both ends, Bam.cpp:596-790)
    const bool bam = spl >= 4 && strcmp(samPath + spl - 4, ".bam") == 0;
    // One aligner's align calls serve one host thread at a time (mT / mG; ga also runs the paired
    // aligner's single-end fallback), and so do its side-stream calls (seed census, CIGARs: mTs /
    // mGs); the two kinds share no stream or buffer, so stage B of a sub-batch overlaps stage A of
    // the next on the device too.
    std::mutex mG, mTown, mGs, mTsOwn;
    std::mutex &mT = ta == ga ? mG : mTown;
    std::mutex &mTs = ta == ga ? mGs : mTsOwn;
    RnaRun Rr{pa, ta, ga, gi, ti, gtf, {R[0], R[1]}, opt, &useful, &mT, &mG, &mTs, &mGs, &C, bam};
    // Sub-batches of the pairs, pipelined: stage A (the GPU aligners) of sub-batch s + 1 runs while
    // stage B (filter, seed census, counts, CIGARs, records) of sub-batch s runs on another thread,
    // its GPU calls on the aligners' side streams.  Every stage keeps the reference's per-pair
    // semantics; records and count events stay in input order across sub-batches.  Each aligner call
    // pays the tail of its slowest pair (a persistent kernel ends with its heaviest reads, even
    // longest-first), so the split is coarse: two halves from 40k pairs up (100k 2 x 150 pairs:
    // 77.0 -> 72.7 ms; three and four sub-batches 93.6 / 100.6 ms, profiles/r05/ab/rna_sub_r05k.txt).
    // SNAPGPU_RNA_SUBBATCH = pairs per sub-batch overrides it.
    uint64_t per = n >= 40000 ? (n + 1) / 2 : (n ? n : 1);
    if (const char *e = getenv("SNAPGPU_RNA_SUBBATCH"); e && atoll(e) > 0) per = (uint64_t)atoll(e);
    const uint64_t S = n ? (n + per - 1) / per : 0;
    std::vector<std::unique_ptr<RnaSub>> subs(S);
    for (uint64_t k = 0; k < S; k++) {
        subs[k].reset(new RnaSub);
        subs[k]->a = k * per;
        subs[k]->b = std::min(n, (k + 1) * per);
    }
    std::mutex qm;
    std::condition_variable cv;
    uint64_t aDone = 0;
    bool stop = false;
    int32_t lastNm = 0;   // BAM NM carry-over, in write order across sub-batches
    std::thread stageB([&] {
        for (uint64_t k = 0; k < S; k++) {
            {
                std::unique_lock<std::mutex> lk(qm);
                cv.wait(lk, [&] { return aDone > k || stop; });
                if (stop && aDone <= k) return;
            }
            RnaSub &X = *subs[k];
            if (X.rc == SNAPGPU_OK) rnaStageB(Rr, X, lastNm);
            if (X.rc != SNAPGPU_OK) {
                std::lock_guard<std::mutex> lk(qm);
                stop = true;
                cv.notify_all();
                return;
            }
        }
    });
    for (uint64_t k = 0; k < S; k++) {
        {
            std::lock_guard<std::mutex> lk(qm);
            if (stop) break;
        }
        rnaStageA(Rr, *subs[k]);
        std::lock_guard<std::mutex> lk(qm);
        aDone = k + 1;
        if (subs[k]->rc != SNAPGPU_OK) stop = true;
        cv.notify_all();
    }
    stageB.join();
    for (auto &x : subs)
        if (x->rc != SNAPGPU_OK) {
            setError(x->err);
            return x->rc;
        }
    // GTFReader::IncrementReadCount for every counted pair, in input order, all or nothing
    {
        const auto t1 = std::chrono::steady_clock::now();
        std::vector<GtfPairQuery> cq;
        for (auto &x : subs) cq.insert(cq.end(), x->cq.begin(), x->cq.end());
        std::vector<uint32_t> contamLocs;
        for (auto &x : subs) contamLocs.insert(contamLocs.end(), x->contamLocs.begin(), x->contamLocs.end());
        if (!contamLocs.empty()) {   // resolved before anything is counted: a bad location counts nothing
            const int rc = contaminantsAddAll(opt->contaminants, contamLocs, false);
            if (rc) return rc;
        }
        if (gtfCountPairs(gtf, cq) >= 0) {
            setError("rna_paired_align: read count for an unknown transcript or gene");
            return SNAPGPU_EFORMAT;
        }
        if (!contamLocs.empty()) contaminantsAddAll(opt->contaminants, contamLocs);   // checked above
        st.countedPairs = cq.size();
        st.countMs += msSince(t1);
    }
    for (auto &x : subs) {
        st.singleHits += x->single; st.multiHits += x->multi; st.notFound += x->notFound;
        st.partialPairs += x->partialPairs; st.partialMatches += x->partialMatches; st.seedRuns += x->seedRuns;
        st.transcriptomeRecords += x->transcriptomeRecords;
        st.alignMs += x->alignMs; st.filterMs += x->filterMs; st.seedMs += x->seedMs; st.countMs += x->countMs;
        st.cigarMs += x->cigarMs; st.writeMs += x->writeMs;
        st.cigarGpuMs += x->cigarGpuMs; st.spliceMs += x->spliceMs;
    }
    if (samPath) {
        const auto t1 = std::chrono::steady_clock::now();
        FILE *f = fopen(samPath, "w");
        if (!f) { setError(std::string("cannot write ") + samPath); return SNAPGPU_EIO; }
        uint64_t hlen = 0;
        const int so = opt->sortOutput ? 1 : 0;   // @HD SO:coordinate (SAMFormat::writeHeader, sorted)
        snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "", nullptr,
                           nullptr, 0, &hlen);
        std::string hdr(hlen, '\0');
        int rc = snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "",
                                    nullptr, &hdr[0], hlen, &hlen);
        if (rc) { fclose(f); return rc; }
        bool ok = true;
        if (bam) {   // BGZF stream: header, then the records (64 KB blocks), then the EOF block
            hdr.resize(strnlen(hdr.data(), hdr.size()));
            const std::string bh = bamHeader(*gi->genome, hdr);
            ok = bgzfWrite(f, bh.data(), bh.size(), false);
            std::string all;
            for (auto &x : subs)
                for (auto &p : x->parts) all += p;
            ok = ok && bgzfWrite(f, all.data(), all.size(), true);
        } else {
            ok = fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
            if (opt->sortOutput) {   // one block: the whole call's records, stable-sorted by location
                std::vector<std::string> all;
                for (auto &x : subs)
                    for (auto &p : x->parts) all.push_back(std::move(p));
                const std::string sorted = samSortRecords(*gi->genome, all);
                ok = ok && fwrite(sorted.data(), 1, sorted.size(), f) == sorted.size();
            } else {
                for (auto &x : subs)
                    for (auto &p : x->parts) ok = ok && fwrite(p.data(), 1, p.size(), f) == p.size();
            }
        }
        ok = (fclose(f) == 0) && ok;
        if (!ok) { setError(std::string("write failed: ") + samPath); return SNAPGPU_EIO; }
        st.writeMs += msSince(t1);
    }
    if (out)
        for (auto &x : subs)
            for (uint64_t i = x->a; i < x->b; i++) {
                const PairOut &r = x->po[i - x->a];
                snapgpu_rna_pair_result_t &o = out[i];
                memset(&o, 0, sizeof(o));
                for (int k = 0; k < 2; k++) {
                    o.status[k] = (uint8_t)r.status[k];
                    o.location[k] = r.status[k] != SNAPGPU_NOT_FOUND ? r.location[k] : kInvalidLocation;
                    o.tlocation[k] = r.tlocation[k];
                    o.direction[k] = (uint8_t)r.direction[k];
                    o.score[k] = r.score[k];
                    o.mapq[k] = r.mapq[k];
                    o.isTranscriptome[k] = r.isTranscriptome[k];
                }
                o.fromAlignTogether = r.fromAlignTogether;
                o.alignedAsPair = r.alignedAsPair;
                o.useful = useful[i];
            }
    st.subBatches = S;
    st.wallMs = msSince(w0);
    if (stats) *stats = st;
    return SNAPGPU_OK;
}

}  // extern "C"

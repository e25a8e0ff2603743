// single.cpp -- the single-end RNA product path: `snap-rna single` over a
// whole batch, with both BaseAligner::AlignRead calls per read and the CIGARs on the GPU.
//
// SingleAlignerContext::runIterationThread (SingleAligner.cpp:141-320) handles one read at a
// time: pre-filter, transcriptome AlignRead, genome AlignRead, AlignmentFilter, writeRead.  Here
// each stage runs over the batch: the pre-filter on the host, the two aligners as batched GPU
// calls (snapgpu_align_batch), AlignmentFilter::AddAlignment / FilterSingle on host threads,
// the CIGARs of all records as two GPU batches (genome and transcriptome), the lines on host
// threads, written in input order.
#include "internal.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_map>
#include <string>
#include <thread>
#include <vector>


namespace snapgpu {
struct GtfTranscript;
const GtfTranscript *gtfTranscript(const snapgpu_gtf_t *g, const std::string &id);
const std::string &gtfTranscriptChr(const GtfTranscript *t);
uint32_t gtfGenomicPosition(const GtfTranscript *t, uint32_t pos, uint32_t span);
bool gtfSpliceCigar(const GtfTranscript *t, uint32_t pos, const std::vector<std::pair<uint32_t, char>> &tokens,
                    std::string &out);
void gtfCountSingle(snapgpu_gtf_t *g, const std::string &transcriptId);
uint32_t *gtfGeneCounter(snapgpu_gtf_t *g, const std::string &transcriptId);
}  // namespace snapgpu

using namespace snapgpu;

namespace {

double msSince(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Genome::getPieceAtLocation (Genome.cpp:356-374); -1 before the first piece
int pieceAt(const Genome &g, uint32_t loc) {
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

// Alignment (AlignmentFilter.h:41-70), the fields FilterSingle reads.  The names point into storage
// that outlives the call (the genome's and the transcriptome's piece names, the GTF's chromosome
// names), so a read's filter allocates nothing.
struct Alignment {
    uint32_t location = 0;
    int direction = 0;
    int score = 0;
    const std::string *rname = nullptr, *transcriptId = nullptr;
    uint32_t pos = 0;
    bool isTranscriptome = false;
};

// (no default member initialisers: a 1M-read call allocates these uninitialised; filterSingle writes
// every field of every read's entry)
struct FilterOut {
    const std::string *countTranscript;   // GTFReader::IncrementReadCount (:261, :291)
    int result;
    uint32_t location, tlocation;
    int direction, score, mapq;
    bool isTranscriptome;
    static FilterOut notFound() { return FilterOut{nullptr, SNAPGPU_NOT_FOUND, 0, 0, 0, 0, 0, false}; }
};

struct Ctx {
    const Genome *genome, *transcriptome;
    snapgpu_gtf_t *gtf;
    std::map<std::string, uint32_t> pieceByName;   // Genome::getOffsetOfPiece (Genome.cpp:317-345)
    uint32_t maxDist, confDiff;
};

// AlignmentFilter's mate-0 map (AlignmentFilter.cpp:113-214), keyed by rname + '_' + pos: a single-end
// read adds at most two alignments (transcriptome, then genome), so the map is two slots, and its
// iteration order -- the order FilterSingle sorts from -- is the keys' std::string order.
struct Mate0 {
    Alignment a[2];
    int n = 0;
};
// key(x) < key(y) as std::string compares rname + "_" + decimal pos (char_traits<char>: unsigned bytes)
bool keyLess(const Alignment &x, const Alignment &y) {
    char kx[320], ky[320];
    const int lx = snprintf(kx, sizeof kx, "%s_%u", x.rname->c_str(), x.pos);
    const int ly = snprintf(ky, sizeof ky, "%s_%u", y.rname->c_str(), y.pos);
    if (lx < (int)sizeof kx && ly < (int)sizeof ky) {
        const int c = memcmp(kx, ky, (size_t)std::min(lx, ly));
        return c != 0 ? c < 0 : lx < ly;
    }
    return *x.rname + '_' + std::to_string(x.pos) < *y.rname + '_' + std::to_string(y.pos);   // (names > 300 bytes)
}

// AlignmentFilter::AddAlignment + HashAlignment (AlignmentFilter.cpp:113-214), mate 0
int addAlignment(const Ctx &C, Mate0 &mate0, uint32_t location, int direction, int score, bool isTranscriptome,
                 uint32_t readLen, std::string *err) {
    if (score > (int)C.maxDist) return -1;   // `score > maxDist`: unsigned comparison in the reference
    static const std::string kStar = "*";
    const std::string *rname = &kStar, *tid = nullptr;
    uint32_t pos = 0;
    if (location != kInvalidLocation) {
        const Genome &g = isTranscriptome ? *C.transcriptome : *C.genome;
        const int p = pieceAt(g, location);
        if (p < 0) return 0;   // before the first piece (the reference dereferences NULL)
        rname = &g.pieceNames[p];
        pos = location - g.pieceOffsets[p] + 1;
        if (isTranscriptome) {
            const GtfTranscript *t = gtfTranscript(C.gtf, *rname);
            if (!t) { *err = "No transcript " + *rname; return -2; }   // GTFReader::GetTranscript exits
            tid = rname;
            rname = &gtfTranscriptChr(t);
            pos = gtfGenomicPosition(t, pos, readLen);
        }
    }
    if (pos == 0) return 0;
    Alignment a;
    a.location = location; a.direction = direction; a.score = score; a.rname = rname; a.pos = pos;
    a.isTranscriptome = isTranscriptome;
    a.transcriptId = tid;
    for (int i = 0; i < mate0.n; i++) {
        Alignment &o = mate0.a[i];
        if (o.pos == pos && *o.rname == *rname) {   // the same key
            if (a.score < o.score) o = a;
            else if (a.score == o.score && a.isTranscriptome) o = a;
            return 0;
        }
    }
    mate0.a[mate0.n++] = a;
    return 0;
}

// AlignmentFilter::FilterSingle (AlignmentFilter.cpp:216-300)
bool filterSingle(const Ctx &C, Mate0 &mate0, FilterOut &o, std::string *err) {
    if (mate0.n == 2 && keyLess(mate0.a[1], mate0.a[0])) std::swap(mate0.a[0], mate0.a[1]);   // map order
    const Alignment *al[2];
    int na = 0;
    for (int i = 0; i < mate0.n; i++)
        if (!(mate0.a[i].score > (int)C.maxDist)) al[na++] = &mate0.a[i];
    if (na == 0) { o = FilterOut::notFound(); return true; }
    if (na == 2 && al[1]->score < al[0]->score) std::swap(al[0], al[1]);   // std::sort of two: stable
    const Alignment &a = *al[0];
    if (a.isTranscriptome) {
        auto po = C.pieceByName.find(*a.rname);
        if (po == C.pieceByName.end()) { *err = "chromosome " + *a.rname + " not in the genome"; return false; }
        o.tlocation = a.location;
        o.location = po->second + a.pos - 1;
    } else {
        o.location = a.location;
        o.tlocation = 0;
    }
    o.direction = a.direction;
    o.score = a.score;
    o.isTranscriptome = a.isTranscriptome;
    o.countTranscript = nullptr;
    if (na == 1 || (uint32_t)(al[1]->score - al[0]->score) >= C.confDiff) {
        o.mapq = 70;   // min(maxMAPQ, genome_mapq), both 70
        o.result = SNAPGPU_SINGLE_HIT;
        if (a.isTranscriptome) o.countTranscript = a.transcriptId;
    } else {
        o.mapq = 1;
        o.result = SNAPGPU_MULTIPLE_HITS;
    }
    return true;
}

template <class F>
void parallel(uint64_t n, F &&f) {
    const unsigned nt = n < 4096 ? 1u : hostThreads(16);
    if (nt == 1) { f(0u, (uint64_t)0, n); return; }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
    for (auto &x : th) x.join();
}

}  // namespace

extern "C" {

void snapgpu_single_options_default(snapgpu_single_options_t *o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->clipping = 3;                  // AlignerOptions.cpp:33-85
    o->confDiff = 2;
    o->maxDist = 14;
    o->minPercentAbovePhred = 90.0f;
    o->minPhred = 20;
    o->phredOffset = 33;
    o->useM = 0;
    o->readGroup = "FASTQ";
    o->commandLine = "";
    o->version = "";
}

int snapgpu_single_align(snapgpu_aligner_t *ga, snapgpu_aligner_t *ta, snapgpu_gtf_t *gtf,
                         snapgpu_reads_t *reads, const snapgpu_single_options_t *opt, const char *samPath,
                         snapgpu_single_stats_t *stats) {
    const auto w0 = std::chrono::steady_clock::now();
    if (!ga || !ta || !gtf || !reads || !opt || !samPath) { setError("single_align: null argument"); return SNAPGPU_EINVAL; }
    if (!reads->ids) { setError("single_align: the reads carry no ids (use snapgpu_reads_from_fastq)"); return SNAPGPU_EINVAL; }
    // BAM output when the path ends in ".bam" (AlignerOptions: "SAM or BAM format, depending on the
    // file extension"); sorted BAM (+ BAMIndexSupplier's .bai) is not built -- refused before any
    // alignment or counting, so a refused call leaves the caller's GTF and contamination counts alone
    const size_t pl = strlen(samPath);
    const bool bam = pl >= 4 && strcmp(samPath + pl - 4, ".bam") == 0;
    if (bam && opt->sortOutput) {
        setError("single_align: sorted output is built for SAM only");
        return SNAPGPU_EUNSUPPORTED;
    }
    const snapgpu_index_t *gi = snapgpu_aligner_index(ga), *ti = snapgpu_aligner_index(ta);
    snapgpu_single_stats_t st{};
    int rc = snapgpu_reads_clip(reads, opt->clipping, nullptr, nullptr);   // FASTQReader (FASTQ.cpp:250)
    if (rc) return rc;
    const uint64_t n = reads->n;
    st.totalReads = n;
    // pre-filter (SingleAligner.cpp:247-257): Read::qualityFilter, length, Read::countOfNs
    std::vector<uint8_t> useful(n, 0);
    parallel(n, [&](unsigned, uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            const char *q = reads->quals + reads->offsets[i], *d = reads->bases + reads->offsets[i];
            const uint32_t len = reads->lengths[i];
            unsigned count = 0, ns = 0;
            for (uint32_t j = 0; j < len; j++) {
                if ((unsigned)(int)q[j] - opt->phredOffset >= opt->minPhred) count++;   // Read.h:425
                ns += d[j] == 'N' || d[j] == 'n';                                     // IS_N (Tables.cpp:32-33)
            }
            const bool quality = ((float)count / (float)len) * 100.f >= opt->minPercentAbovePhred;
            useful[i] = !(len < 50 || ns > opt->maxDist || !quality);
        }
    });
    std::vector<uint64_t> ui;   // useful read -> batch index
    for (uint64_t i = 0; i < n; i++) if (useful[i]) ui.push_back(i);
    const uint64_t nu = ui.size();
    st.usefulReads = nu;
    std::vector<uint64_t> uo(nu + 1);
    std::vector<uint32_t> ul(nu + 1);
    for (uint64_t j = 0; j < nu; j++) { uo[j] = reads->offsets[ui[j]]; ul[j] = reads->lengths[ui[j]]; }
    snapgpu_reads_t *ub = readsView(reads, nu, uo.data(), ul.data());   // the useful reads, no copy
    if (!ub) return SNAPGPU_ENOMEM;
    // per-read arrays the stages below write in full are left uninitialised (zero-filling the CIGAR
    // op tables of 1M reads was most of the call's preparation)
    std::unique_ptr<snapgpu_result_t[]> tr(new snapgpu_result_t[nu + 1]), gr(new snapgpu_result_t[nu + 1]);
    std::unique_ptr<FilterOut[]> fo(new FilterOut[nu + 1]);
    std::vector<int32_t> ted(nu + 1, -1);   // NM of the transcriptome records
    std::vector<int64_t> uidx(n, -1);
    for (uint64_t j = 0; j < nu; j++) uidx[ui[j]] = (int64_t)j;
    auto fail = [&](int code) { snapgpu_reads_free(ub); return code; };
    Ctx C{gi->genome, ti->genome, gtf, {}, opt->maxDist, opt->confDiff};
    for (size_t p = 0; p < gi->genome->pieceNames.size(); p++) C.pieceByName.insert({gi->genome->pieceNames[p], gi->genome->pieceOffsets[p]});
    // Sub-batches (SNAPGPU_SINGLE_SUBBATCH useful reads each; default two halves from 200k reads, one
    // for BAM and sorted output, whose records are written as one block): stage A aligns sub-batch s
    // (both aligners in flight) on this thread while a stage-B thread runs sub-batch s - 1's filter,
    // CIGARs (the aligners' side streams) and records, and a writer thread writes sub-batch s - 2's
    // records -- the file in input order, the counts of the whole call applied at the end, all or
    // nothing.
    uint64_t sub = nu;
    if (const char *e = getenv("SNAPGPU_SINGLE_SUBBATCH"); e && atoll(e) > 0) sub = (uint64_t)atoll(e);
    else if (nu >= 200000) sub = (nu + 1) / 2;
    if (bam || opt->sortOutput || sub == 0) sub = nu ? nu : 1;
    const uint64_t nSub = nu ? (nu + sub - 1) / sub : 1;
    std::vector<snapgpu_reads_t *> views(nSub, nullptr);
    for (uint64_t b = 0; b < nSub; b++) {
        const uint64_t ja = b * sub, jb = std::min(nu, ja + sub);
        views[b] = readsView(reads, jb - ja, uo.data() + ja, ul.data() + ja);
        if (!views[b]) { for (auto *v : views) snapgpu_reads_free(v); return fail(SNAPGPU_ENOMEM); }
    }
    auto freeViews = [&] { for (auto *&v : views) { snapgpu_reads_free(v); v = nullptr; } };
    st.prepMs = msSince(w0);
    // stage A of sub-batch b: t_aligner then g_aligner (SingleAligner.cpp:270-276), both submitted
    // before either is waited for (their own streams: one's upload and kernels overlap the other's)
    auto stageA = [&](uint64_t b) -> int {
        const uint64_t ja = b * sub, jb = std::min(nu, ja + sub);
        if (jb <= ja) return SNAPGPU_OK;
        snapgpu_reads_t *v = views[b];
        int r;
        if ((r = snapgpu_align_batch_submit(ta, v, tr.get() + ja))) { snapgpu_align_batch_wait(ta); return r; }
        if (ga != ta && (r = snapgpu_align_batch_submit(ga, v, gr.get() + ja))) {
            snapgpu_align_batch_wait(ta);
            snapgpu_align_batch_wait(ga);
            return r;
        }
        const int rt = snapgpu_align_batch_wait(ta);
        const int rg = ga != ta ? snapgpu_align_batch_wait(ga) : SNAPGPU_OK;
        if ((r = rt ? rt : rg)) return r;
        if (ga == ta) r = snapgpu_align_batch(ga, v, gr.get() + ja);   // one aligner for both
        return r;
    };
    // the output file and its header (SAM text; BAM after all records)
    FILE *f = fopen(samPath, "w");
    if (!f) { setError(std::string("cannot write ") + samPath); freeViews(); return fail(SNAPGPU_EIO); }
    uint64_t hlen = 0;
    const int so = opt->sortOutput ? 1 : 0;   // @HD SO:coordinate (SAMFormat::writeHeader, sorted)
    snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "", nullptr,
                       nullptr, 0, &hlen);
    std::string hdr(hlen, '\0');
    if ((rc = snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "",
                                 nullptr, &hdr[0], hlen, &hlen))) { fclose(f); freeViews(); return fail(rc); }
    bool ok = true;
    if (!bam) ok = fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
    std::vector<std::string> allParts;   // BAM / sorted: every record part, written at the end
    // SAM: a sub-batch's records are written by their own thread while the next sub-batch is
    // filtered and formatted (one writer at a time, in sub-batch order)
    std::thread writer;
    bool writeOk = true;
    double writeMs = 0;
    std::vector<uint32_t> contamLocs;    // added with the GTF counts once nothing can fail any more
    std::string errMsg;
    int32_t lastNm = 0;                  // BAM NM carry-over (before any mapped record: the stack's leftover)
    const unsigned nw = n < 4096 ? 1u : hostThreads(16);
    std::vector<uint64_t> cnt(16 * nw, 0);   // thread t's three counters at 16 t: a cache line of their own
    // stage B of sub-batch b (useful reads [ja, jb), input reads [ia, ib))
    std::vector<std::string> splice;   // stage B's current sub-batch: transcriptome CIGARs (compact)
    std::vector<int32_t> spliceAt;     //   and each useful read's index into them (-1: none)
    auto stageB = [&](uint64_t b) -> int {
        const uint64_t ja = b * sub, jb = std::min(nu, ja + sub), m = jb - ja;
        const uint64_t ia = b == 0 ? 0 : ui[ja], ib = b + 1 >= nSub ? n : ui[jb];
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::string> errs(hostThreads(16));
        parallel(m, [&](unsigned t, uint64_t x, uint64_t y) {
            for (uint64_t j = ja + x; j < ja + y && errs[t].empty(); j++) {
                Mate0 mate0;
                // AlignmentFilter (AlignmentFilter.cpp:107-109); AddAlignment uses read1 = the read
                if (addAlignment(C, mate0, tr[j].location, tr[j].direction, tr[j].score, true, ul[j], &errs[t]) == -2) break;
                if (addAlignment(C, mate0, gr[j].location, gr[j].direction, gr[j].score, false, ul[j], &errs[t]) == -2) break;
                if (!filterSingle(C, mate0, fo[j], &errs[t])) break;
            }
        });
        for (auto &e : errs) if (!e.empty()) { errMsg = "single_align: " + e; return SNAPGPU_EFORMAT; }
        // -ct (SingleAligner.cpp:282-293): the reads still NotFound through the contamination
        // BaseAligner, one GPU batch; every read it aligns counts its contig (ContaminationFilter)
        if (opt->contaminationAligner && opt->contaminants && m) {
            std::vector<uint64_t> co;
            std::vector<uint32_t> cl;
            for (uint64_t j = ja; j < jb; j++)
                if (fo[j].result == SNAPGPU_NOT_FOUND) { co.push_back(uo[j]); cl.push_back(ul[j]); }
            if (!co.empty()) {
                snapgpu_reads_t *cb = readsView(reads, co.size(), co.data(), cl.data());
                if (!cb) return SNAPGPU_ENOMEM;
                std::vector<snapgpu_result_t> cr(co.size());
                const int r = snapgpu_align_batch(opt->contaminationAligner, cb, cr.data());
                snapgpu_reads_free(cb);
                if (r) return r;
                for (auto &x : cr)
                    if (x.result != SNAPGPU_NOT_FOUND) contamLocs.push_back(x.location);
            }
        }
        st.filterMs += msSince(t0);
        // CIGARs on the GPU: genome records at the filter's location (NotFound keeps location 0 and
        // the forward read, SAM.cpp:1040-1048), transcriptome records on the transcriptome at tlocation
        t0 = std::chrono::steady_clock::now();
        const int32_t *ged = nullptr;   // the genome records' CIGARs, left in the genome aligner's pinned
        const uint32_t *gn = nullptr, *gops = nullptr;   // output buffer (indexed j - ja) until its next call
        if (m) {
            std::vector<uint32_t> gl(m), tl(m);
            std::vector<uint8_t> gd(m), td(m);
            uint64_t nt = 0;
            for (uint64_t j = ja; j < jb; j++) {
                const bool isT = fo[j].result != SNAPGPU_NOT_FOUND && fo[j].isTranscriptome;
                gl[j - ja] = isT ? kInvalidLocation : fo[j].location;
                gd[j - ja] = (uint8_t)(fo[j].result == SNAPGPU_NOT_FOUND ? 0 : fo[j].direction);
                tl[j - ja] = isT ? fo[j].tlocation : kInvalidLocation;
                td[j - ja] = (uint8_t)fo[j].direction;
                nt += isT;
            }
            st.transcriptomeRecords += nt;
            // the transcriptome records only (a compact batch, copied out), and the genome batch over
            // every record (left pinned); on two host threads when the aligners differ (each has its
            // own side stream and buffers)
            std::vector<uint64_t> tj, to;
            std::vector<uint32_t> tlen, tloc;
            std::vector<uint8_t> tdir;
            tj.reserve(nt); to.reserve(nt); tlen.reserve(nt); tloc.reserve(nt); tdir.reserve(nt);
            for (uint64_t j = ja; j < jb; j++)
                if (tl[j - ja] != kInvalidLocation) {
                    tj.push_back(j); to.push_back(uo[j]); tlen.push_back(ul[j]); tloc.push_back(tl[j - ja]);
                    tdir.push_back(td[j - ja]);
                }
            splice.assign(nt, std::string());   // this sub-batch's transcriptome CIGARs, by compact index
            spliceAt.assign(m, -1);
            for (uint64_t k = 0; k < nt; k++) spliceAt[tj[k] - ja] = (int32_t)k;
            std::vector<int32_t> tedc(nt + 1, -1);
            std::vector<uint32_t> tnc(nt + 1, 0);
            std::unique_ptr<uint32_t[]> topsc(new uint32_t[(nt + 1) * SNAPGPU_CIGAR_MAX_OPS]);
            const char *const bb[2] = {reads->bases, reads->bases};
            int rcT = SNAPGPU_OK, rcG = SNAPGPU_OK;
            auto runT = [&] {
                if (nt) rcT = snapgpu_internal_cigar_view(ta, bb, nullptr, to.data(), tlen.data(), nt, tloc.data(),
                                                          tdir.data(), (int)opt->useM, tedc.data(), tnc.data(), topsc.get());
            };
            auto runG = [&] {
                rcG = snapgpu_internal_cigar_pinned(ga, bb, nullptr, uo.data() + ja, ul.data() + ja, m, gl.data(), gd.data(),
                                                    (int)opt->useM, &ged, &gn, &gops);
            };
            if (ga != ta && nt) {
                std::thread th(runT);
                runG();
                th.join();
            } else {
                runT();   // (first: with one aligner for both, the genome call reuses its output buffer)
                runG();
            }
            if (rcT || rcG) return rcT ? rcT : rcG;
            for (uint64_t k = 0; k < nt; k++) ted[tj[k]] = tedc[k];
            // transcriptome records: computeCigarString's tokens (soft clips around the ops) through
            // insertSpliceJunctions (SAM.cpp:1049-1064); an unsuccessful LV leaves no tokens
            parallel(nt, [&](unsigned, uint64_t x, uint64_t y) {
                std::vector<std::pair<uint32_t, char>> tk;
                static const char kOp[] = "MIDNSHP=X";
                for (uint64_t k = x; k < y; k++) {
                    const uint64_t j = tj[k];
                    tk.clear();
                    const uint64_t i = ui[j];
                    if (tedc[k] >= 0) {
                        const uint32_t full = reads->unclippedLength[i], front = reads->frontClipped[i];
                        const uint32_t back = full - ul[j] - front;
                        const bool rcd = fo[j].direction == SNAPGPU_RC;
                        const uint32_t before = rcd ? back : front, after = rcd ? front : back;
                        if (before) tk.push_back({before, 'S'});
                        for (uint32_t q = 0; q < tnc[k]; q++) {
                            const uint32_t op = topsc[k * SNAPGPU_CIGAR_MAX_OPS + q];
                            tk.push_back({op >> 4, kOp[op & 15]});
                        }
                        if (after) tk.push_back({after, 'S'});
                    }
                    const Genome &tg = *ti->genome;
                    const int p = pieceAt(tg, tl[j - ja]);
                    const GtfTranscript *t = p >= 0 ? gtfTranscript(gtf, tg.pieceNames[p]) : nullptr;
                    if (t) gtfSpliceCigar(t, tl[j - ja] - tg.pieceOffsets[p] + 1, tk, splice[k]);
                }
            });
        }
        st.cigarMs += msSince(t0);
        // lines of input reads [ia, ib) in input order (writeRead, SingleAligner.cpp:322-336; filtered
        // reads :250-254)
        t0 = std::chrono::steady_clock::now();
        const uint64_t nIn = ib - ia;
        const unsigned nt = nIn < 4096 ? 1u : nw;
        std::vector<std::string> parts(nt);
        // BAMFormat::writeRead sets NM only for a record with a location; the others repeat the
        // previous record's value -- a serial pass in output order fixes each record's NM.
        std::vector<int32_t> bamNm;
        if (bam) {
            bamNm.resize(nIn);
            for (uint64_t i = ia; i < ib; i++) {
                const int64_t j = uidx[i];
                if (j >= 0 && fo[j].result != SNAPGPU_NOT_FOUND)
                    lastNm = fo[j].isTranscriptome ? ted[j] : ged[j - ja];
                bamNm[i - ia] = lastNm;
            }
        }
        std::vector<uint8_t> bamBad(nt, 0);
        auto fmt = [&](unsigned t, uint64_t x, uint64_t y) {
            // built in a local string and swapped in at the end: the parts' string headers sit side by
            // side in the vector, and appending through them moved their shared cache lines between
            // the writer threads on every field
            std::string o;
            o.reserve((y - x) * 320);
            for (uint64_t i = ia + x; i < ia + y; i++) {
                SamLine L;
                L.id = reads->ids + reads->idOffsets[i];
                L.idLen = reads->idLengths[i];
                L.front = reads->frontClipped[i];
                L.clippedLen = reads->lengths[i];
                L.fullLen = reads->unclippedLength[i];
                L.bases = reads->bases + reads->offsets[i] - L.front;
                L.quals = reads->quals + reads->offsets[i] - L.front;
                L.rg = opt->readGroup;
                const int64_t j = uidx[i];
                if (j < 0) {   // readWriter->writeRead(read, NotFound, 0, InvalidGenomeLocation, ...)
                    L.result = SNAPGPU_NOT_FOUND;
                    L.loc = kInvalidLocation;
                } else {
                    const FilterOut &fr = fo[j];
                    L.result = fr.result;
                    L.loc = fr.location;
                    L.dir = fr.direction;
                    L.mapq = fr.mapq;
                    if (fr.result != SNAPGPU_NOT_FOUND && fr.isTranscriptome) {
                        L.cigar = &splice[(size_t)spliceAt[j - ja]];
                        L.ed = ted[j];
                    } else {
                        L.ed = ged[j - ja];
                        L.ops = gops + (j - ja) * SNAPGPU_CIGAR_MAX_OPS;
                        L.nOps = gn[j - ja];
                    }
                    // updateStats (SingleAligner.cpp:338-365)
                    cnt[16 * t + (fr.result == SNAPGPU_SINGLE_HIT ? 0 : fr.result == SNAPGPU_MULTIPLE_HITS ? 1 : 2)]++;
                }
                if (bam && L.result == SNAPGPU_NOT_FOUND) L.loc = kInvalidLocation;   // BAM: FilterSingle's NotFound
                                                                                   // location 0 gives no CIGAR, bin (-1, 0)
                if (!bam) samAppendLine(o, *gi->genome, L);
                else if (!bamAppendRecord(o, *gi->genome, L, bamNm[i - ia])) bamBad[t] = 1;
            }
            parts[t].swap(o);
        };
        if (nt == 1) fmt(0, 0, nIn);
        else {
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nt; t++) th.emplace_back(fmt, t, nIn * t / nt, nIn * (t + 1) / nt);
            for (auto &x : th) x.join();
        }
        for (unsigned t = 0; t < nt; t++)
            if (bamBad[t]) {
                errMsg = "single_align: BAM record not written (QNAME longer than 254 characters, Bam.cpp:723-726)";
                return SNAPGPU_EINVAL;
            }
        st.formatMs += msSince(t0);
        t0 = std::chrono::steady_clock::now();
        if (bam || opt->sortOutput) {
            for (auto &p : parts) allParts.push_back(std::move(p));
        } else {
            // one sequential write per sub-batch, in order, on the writer thread (the file output is
            // ~50 ms of a 1M-read call on the box's tmpfs; parallel pwrites and a shared mapping filled
            // by the formatting threads measured slower, profiles/r06/ab/single_write_r06h.txt)
            if (writer.joinable()) writer.join();
            writer = std::thread([&, ps = std::move(parts)]() {
                const auto tw = std::chrono::steady_clock::now();
                for (auto &p : ps) writeOk = writeOk && fwrite(p.data(), 1, p.size(), f) == p.size();
                writeMs += msSince(tw);
            });
        }
        st.ioMs += msSince(t0);
        return SNAPGPU_OK;
    };
    // the pipeline: A(0); then A(b + 1) here while B(b) runs on the stage-B thread
    int rcA = SNAPGPU_OK, rcB = SNAPGPU_OK;
    {
        auto ta0 = std::chrono::steady_clock::now();
        rcA = stageA(0);
        st.alignMs += msSince(ta0);
        for (uint64_t b = 0; b < nSub && rcA == SNAPGPU_OK && rcB == SNAPGPU_OK; b++) {
            std::thread tb([&, b] { rcB = stageB(b); });
            if (b + 1 < nSub) {
                auto t1 = std::chrono::steady_clock::now();
                rcA = stageA(b + 1);
                st.alignMs += msSince(t1);
            }
            tb.join();
        }
        if (writer.joinable()) writer.join();
        ok = ok && writeOk;
        st.ioMs += writeMs;
    }
    if (rcA || rcB) {
        fclose(f);
        freeViews();
        if (!errMsg.empty()) setError(errMsg);
        return fail(rcA ? rcA : rcB);
    }
    for (unsigned t = 0; t < nw; t++) { st.singleHits += cnt[16 * t]; st.multiHits += cnt[16 * t + 1]; st.notFound += cnt[16 * t + 2]; }
    auto t0 = std::chrono::steady_clock::now();
    if (bam) {   // BGZF stream: header, then the records (64 KB blocks), then the EOF block
        hdr.resize(strnlen(hdr.data(), hdr.size()));
        const std::string bh = bamHeader(*gi->genome, hdr);
        ok = bgzfWrite(f, bh.data(), bh.size(), false);
        std::string all;
        for (auto &p : allParts) all += p;
        ok = ok && bgzfWrite(f, all.data(), all.size(), true);
    } else if (opt->sortOutput) {
        const std::string sorted = samSortRecords(*gi->genome, allParts);
        ok = ok && fwrite(sorted.data(), 1, sorted.size(), f) == sorted.size();
    }
    ok = (fclose(f) == 0) && ok;
    st.ioMs += msSince(t0);
    freeViews();
    if (!ok) { setError(std::string("write failed: ") + samPath); return fail(SNAPGPU_EIO); }
    // the call's counts, all or nothing: gene read counts (FilterSingle :260-262, :290-292) and
    // the -ct contaminants (ContaminationFilter::AddAlignment)
    if (!contamLocs.empty() && (rc = contaminantsAddAll(opt->contaminants, contamLocs))) return fail(rc);
    {   // (each transcript's gene counter resolved once: the names are the transcriptome's piece names)
        std::unordered_map<const std::string *, uint32_t *> ctr;
        for (uint64_t j = 0; j < nu; j++)
            if (const std::string *tid = fo[j].countTranscript) {
                auto it = ctr.find(tid);
                if (it == ctr.end()) it = ctr.emplace(tid, gtfGeneCounter(gtf, *tid)).first;
                if (it->second) (*it->second)++;
            }
    }
    st.writeMs = st.formatMs + st.ioMs;
    st.wallMs = msSince(w0);
    if (stats) *stats = st;
    snapgpu_reads_free(ub);
    return SNAPGPU_OK;
}

}  // extern "C"

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

// Alignment (AlignmentFilter.h:41-70), the fields FilterSingle reads
struct Alignment {
    uint32_t location = 0;
    int direction = 0;
    int score = 0;
    std::string rname, transcriptId;
    uint32_t pos = 0;
    bool isTranscriptome = false;
    bool operator<(const Alignment &r) const { return score < r.score; }   // AlignmentFilter.cpp:55-57
};

struct FilterOut {
    const std::string *countTranscript = nullptr;   // GTFReader::IncrementReadCount (:261, :291)
    int result = SNAPGPU_NOT_FOUND;
    uint32_t location = 0, tlocation = 0;
    int direction = 0, score = 0, mapq = 0;
    bool isTranscriptome = false;
};

struct Ctx {
    const Genome *genome, *transcriptome;
    snapgpu_gtf_t *gtf;
    std::map<std::string, uint32_t> pieceByName;   // Genome::getOffsetOfPiece (Genome.cpp:317-345)
    uint32_t maxDist, confDiff;
};

// AlignmentFilter::AddAlignment + HashAlignment (AlignmentFilter.cpp:113-214), mate 0
int addAlignment(const Ctx &C, std::map<std::string, Alignment> &mate0, uint32_t location, int direction, int score,
                 bool isTranscriptome, uint32_t readLen, std::string *err) {
    if (score > (int)C.maxDist) return -1;   // `score > maxDist`: unsigned comparison in the reference
    std::string rname = "*";
    uint32_t pos = 0;
    std::string tid;
    if (location != kInvalidLocation) {
        const Genome &g = isTranscriptome ? *C.transcriptome : *C.genome;
        const int p = pieceAt(g, location);
        if (p < 0) return 0;   // before the first piece (the reference dereferences NULL)
        rname = g.pieceNames[p];
        pos = location - g.pieceOffsets[p] + 1;
        if (isTranscriptome) {
            const GtfTranscript *t = gtfTranscript(C.gtf, rname);
            if (!t) { *err = "No transcript " + rname; return -2; }   // GTFReader::GetTranscript exits
            tid = rname;
            rname = gtfTranscriptChr(t);
            pos = gtfGenomicPosition(t, pos, readLen);
        }
    }
    if (pos == 0) return 0;
    Alignment a;
    a.location = location; a.direction = direction; a.score = score; a.rname = rname; a.pos = pos;
    a.isTranscriptome = isTranscriptome;
    a.transcriptId = tid;
    const std::string key = rname + '_' + std::to_string(pos);
    auto it = mate0.find(key);
    if (it == mate0.end()) mate0.insert({key, a});
    else if (a.score < it->second.score) it->second = a;
    else if (a.score == it->second.score && a.isTranscriptome) it->second = a;
    return 0;
}

// AlignmentFilter::FilterSingle (AlignmentFilter.cpp:216-300)
bool filterSingle(const Ctx &C, const std::map<std::string, Alignment> &mate0, FilterOut &o, std::string *err,
                  std::string &countTranscript) {
    std::vector<Alignment> al;
    for (auto &m : mate0)
        if (!(m.second.score > (int)C.maxDist)) al.push_back(m.second);
    if (al.empty()) { o = FilterOut(); return true; }
    if (al.size() > 1) std::sort(al.begin(), al.end());
    const Alignment &a = al[0];
    if (a.isTranscriptome) {
        auto po = C.pieceByName.find(a.rname);
        if (po == C.pieceByName.end()) { *err = "chromosome " + a.rname + " not in the genome"; return false; }
        o.tlocation = a.location;
        o.location = po->second + a.pos - 1;
    } else {
        o.location = a.location;
        o.tlocation = 0;
    }
    o.direction = a.direction;
    o.score = a.score;
    o.isTranscriptome = a.isTranscriptome;
    if (al.size() == 1 || (uint32_t)(al[1].score - al[0].score) >= C.confDiff) {
        o.mapq = 70;   // min(maxMAPQ, genome_mapq), both 70
        o.result = SNAPGPU_SINGLE_HIT;
        if (a.isTranscriptome) { countTranscript = a.transcriptId; o.countTranscript = &countTranscript; }
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
    std::vector<snapgpu_result_t> tr(nu + 1), gr(nu + 1);
    std::vector<FilterOut> fo(nu + 1);
    std::vector<std::string> countTid(nu + 1);
    std::vector<int32_t> ged(nu + 1, -1), ted(nu + 1, -1);
    std::vector<uint32_t> gn(nu + 1, 0), tn(nu + 1, 0), gops((nu + 1) * SNAPGPU_CIGAR_MAX_OPS),
        tops((nu + 1) * SNAPGPU_CIGAR_MAX_OPS);
    std::vector<std::string> splice(nu + 1);
    auto fail = [&](int code) { snapgpu_reads_free(ub); return code; };
    auto t0 = std::chrono::steady_clock::now();
    if (nu) {
        // t_aligner then g_aligner (SingleAligner.cpp:270-276), each over the whole batch
        if ((rc = snapgpu_align_batch(ta, ub, tr.data()))) return fail(rc);
        if ((rc = snapgpu_align_batch(ga, ub, gr.data()))) return fail(rc);
    }
    st.alignMs = msSince(t0);
    t0 = std::chrono::steady_clock::now();
    Ctx C{gi->genome, ti->genome, gtf, {}, opt->maxDist, opt->confDiff};
    for (size_t p = 0; p < gi->genome->pieceNames.size(); p++) C.pieceByName.insert({gi->genome->pieceNames[p], gi->genome->pieceOffsets[p]});
    std::vector<std::string> errs(hostThreads(16));
    parallel(nu, [&](unsigned t, uint64_t b, uint64_t e) {
        std::map<std::string, Alignment> mate0;
        for (uint64_t j = b; j < e && errs[t].empty(); j++) {
            mate0.clear();
            // AlignmentFilter (AlignmentFilter.cpp:107-109); AddAlignment uses read1 = the read
            if (addAlignment(C, mate0, tr[j].location, tr[j].direction, tr[j].score, true, ul[j], &errs[t]) == -2) break;
            if (addAlignment(C, mate0, gr[j].location, gr[j].direction, gr[j].score, false, ul[j], &errs[t]) == -2) break;
            if (!filterSingle(C, mate0, fo[j], &errs[t], countTid[j])) break;
        }
    });
    for (auto &e : errs) if (!e.empty()) { setError("single_align: " + e); return fail(SNAPGPU_EFORMAT); }
    // -ct (SingleAligner.cpp:282-293): the reads still NotFound through the contamination
    // BaseAligner, one GPU batch; every read it aligns counts its contig (ContaminationFilter)
    std::vector<uint32_t> contamLocs;   // added with the GTF counts once nothing can fail any more
    if (opt->contaminationAligner && opt->contaminants && nu) {
        std::vector<uint64_t> co;
        std::vector<uint32_t> cl;
        for (uint64_t j = 0; j < nu; j++)
            if (fo[j].result == SNAPGPU_NOT_FOUND) { co.push_back(uo[j]); cl.push_back(ul[j]); }
        if (!co.empty()) {
            snapgpu_reads_t *cb = readsView(reads, co.size(), co.data(), cl.data());
            if (!cb) return fail(SNAPGPU_ENOMEM);
            std::vector<snapgpu_result_t> cr(co.size());
            rc = snapgpu_align_batch(opt->contaminationAligner, cb, cr.data());
            snapgpu_reads_free(cb);
            if (rc) return fail(rc);
            for (auto &r : cr)
                if (r.result != SNAPGPU_NOT_FOUND) contamLocs.push_back(r.location);
        }
    }
    st.filterMs = msSince(t0);
    // CIGARs on the GPU: genome records at the filter's location (NotFound keeps location 0 and
    // the forward read, SAM.cpp:1040-1048), transcriptome records on the transcriptome at tlocation
    t0 = std::chrono::steady_clock::now();
    if (nu) {
        std::vector<uint32_t> gl(nu), tl(nu);
        std::vector<uint8_t> gd(nu), td(nu);
        uint64_t nt = 0;
        for (uint64_t j = 0; j < nu; j++) {
            const bool isT = fo[j].result != SNAPGPU_NOT_FOUND && fo[j].isTranscriptome;
            gl[j] = isT ? kInvalidLocation : fo[j].location;
            gd[j] = (uint8_t)(fo[j].result == SNAPGPU_NOT_FOUND ? 0 : fo[j].direction);
            tl[j] = isT ? fo[j].tlocation : kInvalidLocation;
            td[j] = (uint8_t)fo[j].direction;
            nt += isT;
        }
        st.transcriptomeRecords = nt;
        if ((rc = snapgpu_cigar_batch(ga, ub, gl.data(), gd.data(), (int)opt->useM, ged.data(), gn.data(), gops.data())))
            return fail(rc);
        if (nt && (rc = snapgpu_cigar_batch(ta, ub, tl.data(), td.data(), (int)opt->useM, ted.data(), tn.data(), tops.data())))
            return fail(rc);
        // transcriptome records: computeCigarString's tokens (soft clips around the ops) through
        // insertSpliceJunctions (SAM.cpp:1049-1064); an unsuccessful LV leaves no tokens
        parallel(nu, [&](unsigned, uint64_t b, uint64_t e) {
            std::vector<std::pair<uint32_t, char>> tk;
            static const char kOp[] = "MIDNSHP=X";
            for (uint64_t j = b; j < e; j++) {
                if (tl[j] == kInvalidLocation) continue;
                tk.clear();
                const uint64_t i = ui[j];
                if (ted[j] >= 0) {
                    const uint32_t full = reads->unclippedLength[i], front = reads->frontClipped[i];
                    const uint32_t back = full - ul[j] - front;
                    const bool rcd = fo[j].direction == SNAPGPU_RC;
                    const uint32_t before = rcd ? back : front, after = rcd ? front : back;
                    if (before) tk.push_back({before, 'S'});
                    for (uint32_t k = 0; k < tn[j]; k++) {
                        const uint32_t op = tops[j * SNAPGPU_CIGAR_MAX_OPS + k];
                        tk.push_back({op >> 4, kOp[op & 15]});
                    }
                    if (after) tk.push_back({after, 'S'});
                }
                const Genome &tg = *ti->genome;
                const int p = pieceAt(tg, tl[j]);
                const GtfTranscript *t = p >= 0 ? gtfTranscript(gtf, tg.pieceNames[p]) : nullptr;
                if (t) gtfSpliceCigar(t, tl[j] - tg.pieceOffsets[p] + 1, tk, splice[j]);
            }
        });
    }
    st.cigarMs = msSince(t0);
    // lines in input order (writeRead, SingleAligner.cpp:322-336; filtered reads :250-254)
    t0 = std::chrono::steady_clock::now();
    std::vector<int64_t> uidx(n, -1);
    for (uint64_t j = 0; j < nu; j++) uidx[ui[j]] = (int64_t)j;
    const unsigned nt = n < 4096 ? 1u : hostThreads(16);
    std::vector<std::string> parts(nt);
    std::vector<uint64_t> cnt(16 * nt, 0);   // thread t's three counters at 16 t: a cache line of their own
    // BAMFormat::writeRead sets NM only for a record with a location; the others repeat the
    // previous record's value -- a serial pass in output order fixes each record's NM.
    std::vector<int32_t> bamNm;
    if (bam) {
        bamNm.resize(n);
        int32_t last = 0;   // before any mapped record the reference writes its stack's leftover
        for (uint64_t i = 0; i < n; i++) {
            const int64_t j = uidx[i];
            if (j >= 0 && fo[j].result != SNAPGPU_NOT_FOUND)
                last = fo[j].isTranscriptome ? ted[j] : ged[j];
            bamNm[i] = last;
        }
    }
    std::vector<uint8_t> bamBad(nt, 0);
    parallel(n, [&](unsigned t, uint64_t b, uint64_t e) {
        // built in a local string and swapped in at the end: the parts' string headers sit side by
        // side in the vector, and appending through them moved their shared cache lines between
        // the writer threads on every field
        std::string o;
        o.reserve((e - b) * 320);
        for (uint64_t i = b; i < e; i++) {
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
                const FilterOut &f = fo[j];
                L.result = f.result;
                L.loc = f.location;
                L.dir = f.direction;
                L.mapq = f.mapq;
                if (f.result != SNAPGPU_NOT_FOUND && f.isTranscriptome) {
                    L.cigar = &splice[j];
                    L.ed = ted[j];
                } else {
                    L.ed = ged[j];
                    L.ops = gops.data() + j * SNAPGPU_CIGAR_MAX_OPS;
                    L.nOps = gn[j];
                }
                // updateStats (SingleAligner.cpp:338-365)
                cnt[16 * t + (f.result == SNAPGPU_SINGLE_HIT ? 0 : f.result == SNAPGPU_MULTIPLE_HITS ? 1 : 2)]++;
            }
            if (bam && L.result == SNAPGPU_NOT_FOUND) L.loc = kInvalidLocation;   // BAM: FilterSingle's NotFound
                                                                               // location 0 gives no CIGAR, bin (-1, 0)
            if (!bam) samAppendLine(o, *gi->genome, L);
            else if (!bamAppendRecord(o, *gi->genome, L, bamNm[i])) bamBad[t] = 1;
        }
        parts[t].swap(o);
    });
    for (unsigned t = 0; t < nt; t++)
        if (bamBad[t]) {
            setError("single_align: BAM record not written (QNAME longer than 254 characters, Bam.cpp:723-726)");
            return fail(SNAPGPU_EINVAL);
        }
    for (unsigned t = 0; t < nt; t++) { st.singleHits += cnt[16 * t]; st.multiHits += cnt[16 * t + 1]; st.notFound += cnt[16 * t + 2]; }
    FILE *f = fopen(samPath, "w");
    if (!f) { setError(std::string("cannot write ") + samPath); return fail(SNAPGPU_EIO); }
    uint64_t hlen = 0;
    const int so = opt->sortOutput ? 1 : 0;   // @HD SO:coordinate (SAMFormat::writeHeader, sorted)
    snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "", nullptr,
                       nullptr, 0, &hlen);
    std::string hdr(hlen, '\0');
    if ((rc = snapgpu_sam_header(gi, so, opt->commandLine ? opt->commandLine : "", opt->version ? opt->version : "",
                                 nullptr, &hdr[0], hlen, &hlen))) { fclose(f); return fail(rc); }
    bool ok = true;
    if (bam) {   // BGZF stream: header, then the records (64 KB blocks), then the EOF block
        hdr.resize(strnlen(hdr.data(), hdr.size()));
        const std::string bh = bamHeader(*gi->genome, hdr);
        ok = bgzfWrite(f, bh.data(), bh.size(), false);
        std::string all;
        for (auto &p : parts) all += p;
        ok = ok && bgzfWrite(f, all.data(), all.size(), true);
    } else {
        ok = fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
        if (opt->sortOutput) {
            const std::string sorted = samSortRecords(*gi->genome, parts);
            ok = ok && fwrite(sorted.data(), 1, sorted.size(), f) == sorted.size();
        } else {
            for (auto &p : parts) ok = ok && fwrite(p.data(), 1, p.size(), f) == p.size();
        }
    }
    ok = (fclose(f) == 0) && ok;
    if (!ok) { setError(std::string("write failed: ") + samPath); return fail(SNAPGPU_EIO); }
    // the call's counts, all or nothing: gene read counts (FilterSingle :260-262, :290-292) and
    // the -ct contaminants (ContaminationFilter::AddAlignment)
    if (!contamLocs.empty() && (rc = contaminantsAddAll(opt->contaminants, contamLocs))) return fail(rc);
    for (uint64_t j = 0; j < nu; j++)
        if (fo[j].countTranscript) gtfCountSingle(gtf, *fo[j].countTranscript);
    st.writeMs = msSince(t0);
    st.wallMs = msSince(w0);
    if (stats) *stats = st;
    snapgpu_reads_free(ub);
    return SNAPGPU_OK;
}

}  // extern "C"

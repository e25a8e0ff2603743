// gtf.cpp -- the annotation side of the RNA product path: GTF exons ->
// transcripts, the transcriptome FASTA the reference indexes, transcript -> genome coordinates
// and the splice-junction CIGAR rewrite of transcriptome alignments.
//
// Restates SNAPLib/GTFReader.cpp (GTFFeature ctor :646-713, Parse :1302-1362, Load :1245-1300,
// GTFTranscript::Process :972-1019, GenomicPosition :1075-1105, Junctions :1107-1138,
// WriteFASTA :1181-1212, BuildTranscriptome :1840-1867) and
// LandauVishkinWithCigar::insertSpliceJunctions (LandauVishkin.cpp:119-250), quirks included:
//   * a transcript's feature list is its exons sorted by start with an "intron" feature between
//     consecutive exons; the transcriptome FASTA writes every feature of that list, introns too
//     (the unspliced span), while GenomicPosition counts exon lengths only;
//   * introns are shared by key chr+start+end across genes and transcripts;
//   * all position arithmetic is unsigned 32-bit, as in the reference.
#include "internal.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace snapgpu {

struct GtfFeature {
    std::string key, chr, feature, geneId, transcriptId;
    uint32_t start = 0, end = 0;
    int type = 0;   // 1 exon, 2 intron (GTFReader.h:49)
    uint32_t readCount = 0;   // GTFFeature::read_count (junction counts of introns)
    std::map<std::string, std::string> attributes;
    uint32_t length() const { return end - start + 1; }   // GTFFeature::Length (unsigned)
    bool attr(const std::string &k, std::string &v) const {
        auto it = attributes.find(k);
        if (it == attributes.end()) return false;
        v = it->second;
        return true;
    }
    std::string geneName() const {
        std::string v;
        if (attr("gene_name", v) || attr("Name", v)) return v;
        return geneId;
    }
};

struct GtfTranscript {
    std::string chr, geneId, transcriptId, transcriptName;
    uint32_t start = 0, end = 0;
    float readCount = 0.f;   // GTFTranscript::read_count (float: 1/n per fragment)
    std::vector<const GtfFeature *> features;   // exon lines, in file order
    std::vector<const GtfFeature *> exons;      // after Process: exons and introns by start
};

struct GtfGene {                                         // GTFGene (GTFReader.h:276-312)
    std::string chr, geneId, geneName;
    uint32_t start = 0, end = 0;
    uint32_t readCount = 0;
    std::set<std::string> transcriptIds;
    std::map<std::string, GtfFeature *> introns;         // GTFGene::features: the introns of its transcripts
};

// Static interval index over every feature (exons and introns), the reference's feature_tree
// (IntervalTree.h): sorted by start, implicit balanced tree with the subtree's largest end kept
// at each node's middle index.  Overlap = closed intervals, as IntervalTree::findOverlapping.
struct FeatureIndex {
    std::vector<const GtfFeature *> iv;
    std::vector<uint32_t> maxEnd;
    uint32_t build(size_t lo, size_t hi) {
        if (lo >= hi) return 0;
        const size_t mid = (lo + hi) / 2;
        uint32_t m = iv[mid]->end;
        m = std::max(m, build(lo, mid));
        m = std::max(m, build(mid + 1, hi));
        maxEnd[mid] = m;
        return m;
    }
    void query(size_t lo, size_t hi, uint32_t qs, uint32_t qe, std::vector<const GtfFeature *> &out) const {
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (maxEnd[mid] < qs) return;
            query(lo, mid, qs, qe, out);
            if (iv[mid]->start > qe) return;
            if (iv[mid]->end >= qs) out.push_back(iv[mid]);
            lo = mid + 1;
        }
    }
};

struct Gtf {
    std::map<std::string, GtfFeature> features;          // feature_map (keys stable: pointers stay valid)
    std::map<std::string, GtfTranscript> transcripts;    // transcript_map
    std::map<std::string, GtfGene> genes;                // gene_map
    FeatureIndex featureIndex;
};

// GTFFeature::GTFFeature(string line) (GTFReader.cpp:646-713): strtok on '\'' and '\t' for the
// eight columns, then "key value;" pairs split on " =" / ";" with quotes removed.
static bool parseFeature(const std::string &line, GtfFeature &f) {
    std::vector<char> buf(line.begin(), line.end());
    buf.push_back(0);
    char *save = nullptr;
    const char *d = "'\t'";
    char *p = strtok_r(buf.data(), d, &save);
    if (!p) return false;
    f.chr = p;
    f.key = p;
    if (!(p = strtok_r(nullptr, d, &save))) return false;          // source
    if (!(p = strtok_r(nullptr, d, &save))) return false;
    f.feature = p;
    if (!(p = strtok_r(nullptr, d, &save))) return false;
    f.start = (uint32_t)atoi(p);
    f.key += p;
    if (!(p = strtok_r(nullptr, d, &save))) return false;
    f.end = (uint32_t)atoi(p);
    f.key += p;
    if (!(p = strtok_r(nullptr, d, &save))) return false;          // score
    if (!(p = strtok_r(nullptr, d, &save))) return false;          // strand
    if (!(p = strtok_r(nullptr, d, &save))) return false;          // frame
    for (;;) {
        char *k = strtok_r(nullptr, " =", &save);
        if (!k) break;
        char *v = strtok_r(nullptr, ";", &save);
        if (!v) break;   // the reference would construct a std::string from NULL here
        std::string value = v;
        value.erase(std::remove(value.begin(), value.end(), '"'), value.end());
        f.attributes.insert({k, value});
    }
    if (f.feature == "exon") f.type = 1;
    std::string v;
    if (f.attr("gene_id", v) || f.attr("Parent", v)) f.geneId = v;
    else f.geneId = "Unknown";
    f.transcriptId = f.attr("transcript_id", v) ? v : f.geneId;
    f.key = f.geneId + f.key;
    return true;
}

static std::string u32s(uint32_t x) { return std::to_string(x); }   // ToString (GTFReader.h:398-403)

}  // namespace snapgpu

using namespace snapgpu;

struct snapgpu_gtf : snapgpu::Gtf {};

extern "C" {

snapgpu_gtf_t *snapgpu_gtf_load(const char *path) {
    std::ifstream in(path);
    if (!in.is_open()) { setError(std::string("cannot open GTF ") + path); return nullptr; }
    auto *g = new snapgpu_gtf_t();
    // GTFReader::Load (GTFReader.cpp:1245-1300): getline until eof (a last line without '\n'
    // is not parsed), Parse per line
    std::string line;
    std::getline(in, line, '\n');
    while (!in.eof()) {
        if (!line.empty() && line[0] != '#') {
            GtfFeature f;
            if (parseFeature(line, f) && f.feature == "exon") {   // GTFReader::Parse: exons only
                auto fp = g->features.insert({f.key, f}).first;
                GtfFeature *fe = &fp->second;
                auto tp = g->transcripts.find(f.transcriptId);
                if (tp == g->transcripts.end()) {
                    GtfTranscript t;
                    t.chr = f.chr; t.geneId = f.geneId; t.transcriptId = f.transcriptId;
                    std::string tn;
                    t.transcriptName = f.attr("transcript_name", tn) ? tn : f.transcriptId;   // TranscriptName :728-736
                    t.start = f.start; t.end = f.end;
                    t.features.push_back(fe);
                    g->transcripts.insert({f.transcriptId, t});
                } else {
                    tp->second.features.push_back(fe);
                    tp->second.start = std::min(tp->second.start, f.start);   // UpdateBoundaries
                    tp->second.end = std::max(tp->second.end, f.end);
                }
                auto gp = g->genes.find(f.geneId);
                if (gp == g->genes.end()) {   // GTFGene(chr, gene_id, start, end, GeneName) of the first exon
                    GtfGene ge;
                    ge.chr = f.chr; ge.geneId = f.geneId; ge.geneName = f.geneName();
                    ge.start = f.start; ge.end = f.end;
                    ge.transcriptIds.insert(f.transcriptId);
                    g->genes.insert({f.geneId, ge});
                } else {
                    gp->second.transcriptIds.insert(f.transcriptId);
                    gp->second.start = std::min(gp->second.start, f.start);   // GTFGene::UpdateBoundaries
                    gp->second.end = std::max(gp->second.end, f.end);
                }
            }
        }
        std::getline(in, line, '\n');
    }
    // genes in gene_id order, each gene's transcripts in id order: GTFTranscript::Process
    for (auto &gene : g->genes)
        for (auto &tid : gene.second.transcriptIds) {
            GtfTranscript &t = g->transcripts[tid];
            std::sort(t.features.begin(), t.features.end(),
                      [](const GtfFeature *a, const GtfFeature *b) { return a->start < b->start; });
            const GtfFeature *prev = nullptr;
            for (const GtfFeature *cur : t.features) {
                if (cur->type != 1) continue;
                if (prev) {
                    GtfFeature intron = *cur;
                    intron.feature = "intron";
                    intron.start = prev->end + 1;
                    intron.end = cur->start - 1;
                    intron.key = intron.chr + u32s(intron.start) + u32s(intron.end);
                    intron.type = 2;
                    auto ip = g->features.insert({intron.key, intron}).first;   // shared when present
                    gene.second.introns.insert({intron.key, &ip->second});
                    t.exons.push_back(&ip->second);
                }
                t.exons.push_back(cur);
                prev = cur;
            }
        }
    // feature_tree over every feature, in feature_map order before the sort (Load :1275-1280)
    FeatureIndex &fi = g->featureIndex;
    for (auto &f : g->features) fi.iv.push_back(&f.second);
    std::stable_sort(fi.iv.begin(), fi.iv.end(), [](const GtfFeature *a, const GtfFeature *b) { return a->start < b->start; });
    fi.maxEnd.assign(fi.iv.size(), 0);
    fi.build(0, fi.iv.size());
    return g;
}

void snapgpu_gtf_free(snapgpu_gtf_t *g) { delete g; }

int snapgpu_gtf_counts(const snapgpu_gtf_t *g, uint32_t *nFeatures, uint32_t *nTranscripts, uint32_t *nGenes) {
    if (!g) return SNAPGPU_EINVAL;
    if (nFeatures) *nFeatures = (uint32_t)g->features.size();
    if (nTranscripts) *nTranscripts = (uint32_t)g->transcripts.size();
    if (nGenes) *nGenes = (uint32_t)g->genes.size();
    return SNAPGPU_OK;
}

// GTFReader::BuildTranscriptome / GTFTranscript::WriteFASTA: every transcript in id order as
// ">id\n" + the genome bytes of each feature of its list (exons and introns) + "\n".
int snapgpu_gtf_write_transcriptome(const snapgpu_gtf_t *g, const snapgpu_genome_t *genome, const char *path) {
    if (!g || !genome || !path) return SNAPGPU_EINVAL;
    FILE *f = fopen(path, "w");
    if (!f) { setError(std::string("cannot write ") + path); return SNAPGPU_EIO; }
    std::map<std::string, uint32_t> pieceOffset;
    for (size_t i = 0; i < genome->pieceNames.size(); i++) pieceOffset.insert({genome->pieceNames[i], genome->pieceOffsets[i]});
    const char *b = genome->bases();
    int rc = SNAPGPU_OK;
    for (auto &tp : g->transcripts) {
        const GtfTranscript &t = tp.second;
        auto po = pieceOffset.find(t.chr);
        if (po == pieceOffset.end()) continue;   // "chromosome ... not found in the genome file": skipped
        std::string seq;
        for (const GtfFeature *x : t.exons) {
            const uint64_t at = (uint64_t)x->start + po->second - 1, len = x->length();
            // Genome::getSubstring must serve the whole feature (the reference exits otherwise)
            if (at > genome->nBases || at + len > (uint64_t)genome->nBases + 100) {
                setError("transcript " + t.transcriptId + " exceeds its chromosome");
                rc = SNAPGPU_EFORMAT;
                break;
            }
            seq.append(b + at, len);
        }
        if (rc) break;
        fprintf(f, ">%s\n%s\n", t.transcriptId.c_str(), seq.c_str());
    }
    if (fclose(f) != 0 && rc == SNAPGPU_OK) rc = SNAPGPU_EIO;
    return rc;
}

}  // extern "C"

namespace snapgpu {

const GtfTranscript *gtfTranscript(const snapgpu_gtf_t *g, const std::string &id) {
    auto it = g->transcripts.find(id);
    return it == g->transcripts.end() ? nullptr : &it->second;
}

const std::string &gtfTranscriptChr(const GtfTranscript *t) { return t->chr; }

// GTFTranscript::GenomicPosition (GTFReader.cpp:1075-1105): 1-based transcript position ->
// 1-based genomic position over the exons only; 0 if the span runs past the transcript end.
uint32_t gtfGenomicPosition(const GtfTranscript *t, uint32_t pos, uint32_t span) {
    for (const GtfFeature *x : t->exons) {
        if (x->type != 1) continue;
        if (pos > x->length()) pos -= x->length();
        else {
            const uint32_t gp = x->start + pos - 1;
            if (gp + span > t->end) return 0;
            return gp;
        }
    }
    return 0;
}

// GTFTranscript::Junctions (GTFReader.cpp:1107-1138)
static void junctions(const GtfTranscript *t, uint32_t pos, uint32_t span,
                      std::vector<std::pair<uint32_t, const GtfFeature *>> &out) {
    uint32_t cur = 0;
    const uint32_t endPos = pos + span;
    for (const GtfFeature *x : t->exons) {
        if (x->type == 1) cur += x->length();
        if (pos <= cur) {
            if (x->type == 2) out.push_back({cur + 1, x});
            else if (x->type == 1 && cur >= endPos) return;
        }
    }
}

// LandauVishkinWithCigar::insertSpliceJunctions (LandauVishkin.cpp:119-250) in the
// COMPACT_CIGAR_STRING form: tokens = (count, op) of the transcriptome CIGAR (soft clips
// included); 'N' runs are inserted where a non-I/S operator crosses a junction.
bool gtfSpliceCigar(const GtfTranscript *t, uint32_t pos, const std::vector<std::pair<uint32_t, char>> &tokens,
                    std::string &out) {
    out.clear();
    auto put = [&](uint32_t count, char op) {
        if ((int)count <= 0) return;   // writeCigar: nothing for count <= 0 (an int parameter)
        out += std::to_string((int)count);
        out += op;
    };
    uint32_t prev = pos, current = pos;
    std::vector<std::pair<uint32_t, const GtfFeature *>> js;
    for (auto &tk : tokens) {
        const uint32_t length = tk.first;
        const char op = tk.second;
        if (op == 'I' || op == 'S') { put(length, op); continue; }
        current += length - 1;
        js.clear();
        junctions(t, prev, length, js);
        if (!js.empty()) {
            uint32_t remainder = length;
            for (auto &j : js) {
                if (j.first == pos) continue;   // the read starts on the junction
                const int step = (int)(j.first - prev);
                remainder = remainder - (uint32_t)step;
                if (step > 0) put((uint32_t)step, op);
                put(j.second->length(), 'N');
                prev = prev + (uint32_t)step;
            }
            if (remainder > 0) put(remainder, op);
        } else {
            put(length, op);
        }
        current = current + 1;
        prev = current;
    }
    return true;
}

}  // namespace snapgpu

extern "C" {

int snapgpu_gtf_genomic_position(const snapgpu_gtf_t *g, const char *transcriptId, uint32_t pos, uint32_t span,
                                 uint32_t *out) {
    if (!g || !transcriptId || !out) return SNAPGPU_EINVAL;
    const GtfTranscript *t = gtfTranscript(g, transcriptId);
    if (!t) { setError(std::string("No transcript ") + transcriptId); return SNAPGPU_EINVAL; }
    *out = gtfGenomicPosition(t, pos, span);
    return SNAPGPU_OK;
}

int snapgpu_gtf_splice_cigar(const snapgpu_gtf_t *g, const char *transcriptId, uint32_t pos, uint32_t nTokens,
                             const uint32_t *counts, const char *ops, char *out, uint64_t cap, uint64_t *used) {
    if (!g || !transcriptId || (nTokens && (!counts || !ops)) || !used) return SNAPGPU_EINVAL;
    const GtfTranscript *t = gtfTranscript(g, transcriptId);
    if (!t) { setError(std::string("No transcript ") + transcriptId); return SNAPGPU_EINVAL; }
    std::vector<std::pair<uint32_t, char>> tk;
    for (uint32_t i = 0; i < nTokens; i++) tk.push_back({counts[i], ops[i]});
    std::string s;
    gtfSpliceCigar(t, pos, tk, s);
    *used = s.size();
    if (!out || s.size() + 1 > cap) { setError("splice_cigar: buffer too small"); return SNAPGPU_EINVAL; }
    memcpy(out, s.c_str(), s.size() + 1);
    return SNAPGPU_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ read counts
// GTFReader's per-run counters (GTFFeature / GTFGene / GTFTranscript::IncrementReadCount) and
// the six files GTFReader::WriteReadCounts (GTFReader.cpp:1710-1772) writes after a run.  The
// product paths collect one count event per fragment and apply them in input order: transcript
// counts are float sums of 1/n, whose rounding depends on that order.
namespace snapgpu {

const GtfGene *gtfGene(const snapgpu_gtf_t *g, const std::string &geneId) {
    auto it = g->genes.find(geneId);
    return it == g->genes.end() ? nullptr : &it->second;
}

const std::string &gtfTranscriptGene(const GtfTranscript *t) { return t->geneId; }

// GTFGene::CheckBoundary (GTFReader.cpp:890-902), buffer default 1000 (GTFReader.h:290);
// unsigned arithmetic kept: start - buffer + 1 wraps for genes starting before 1000
bool gtfGeneCheckBoundary(const GtfGene *ge, const std::string &chr, uint32_t pos, uint32_t buffer) {
    if (ge->chr != chr) return false;
    const uint32_t lo = std::max(ge->start - buffer + 1, (uint32_t)1);
    return pos >= lo && pos <= ge->end + buffer;
}

// GTFReader::IncrementReadCount(transcript, ...) single-read form (:1388-1407): the gene only
uint32_t *gtfGeneCounter(snapgpu_gtf_t *g, const std::string &transcriptId);
void gtfCountSingle(snapgpu_gtf_t *g, const std::string &transcriptId) {
    if (uint32_t *c = gtfGeneCounter(g, transcriptId)) (*c)++;
}

// the read counter of the gene of a transcript (GTFReader::IncrementReadCount, single form), or
// nullptr: resolved once per transcript by a caller that counts many reads
uint32_t *gtfGeneCounter(snapgpu_gtf_t *g, const std::string &transcriptId) {
    auto t = g->transcripts.find(transcriptId);
    if (t == g->transcripts.end()) return nullptr;
    auto ge = g->genes.find(t->second.geneId);
    return ge != g->genes.end() ? &ge->second.readCount : nullptr;
}

// the transcripts whose features cover every segment of one read (:1417-1486)
static bool readTranscripts(const snapgpu_gtf_t *g, const std::string &tid, uint32_t tstart, uint32_t start,
                            uint32_t length, std::set<std::string> &ids, std::vector<GtfFeature *> &junc) {
    auto tp = g->transcripts.find(tid);
    if (tp == g->transcripts.end()) return false;   // GetTranscript exits
    const GtfTranscript &t = tp->second;
    std::vector<std::pair<uint32_t, const GtfFeature *>> js;
    junctions(&t, tstart, length, js);
    std::vector<const GtfFeature *> hits;
    auto segment = [&](uint32_t a, uint32_t b) {
        hits.clear();
        g->featureIndex.query(0, g->featureIndex.iv.size(), a, b, hits);
        if (ids.empty()) {
            for (const GtfFeature *f : hits)
                if (f->chr == t.chr) ids.insert(f->transcriptId);
        } else {
            std::set<std::string> keep;
            for (const GtfFeature *f : hits)
                if (f->chr == t.chr && ids.count(f->transcriptId)) keep.insert(f->transcriptId);
            ids.swap(keep);
        }
    };
    for (auto &j : js) {
        junc.push_back(const_cast<GtfFeature *>(j.second));   // the junction's splice count
        const uint32_t len = j.first - tstart;
        segment(start, start + len - 1);
        tstart += len;
        start += len + j.second->length();
        length -= len;
    }
    segment(start, start + length - 1);
    return true;
}

// The counter updates one pair makes (GTFReader::IncrementReadCount, pair form, :1409-1611),
// found without touching any counter: the junctions its reads cross, the transcripts both reads
// are compatible with (in id order) and their gene.  bad: an unknown transcript or gene (the
// reference exits).
struct GtfPairEvent {
    std::vector<GtfFeature *> junc;
    std::vector<GtfTranscript *> tr;
    GtfGene *gene = nullptr;
    bool bad = false;
};

static void pairEvent(const snapgpu_gtf_t *g, const GtfPairQuery &q, GtfPairEvent &ev) {
    std::set<std::string> ids0, ids1;
    if (q.tid0->empty()) return;
    if (!readTranscripts(g, *q.tid0, q.tstart0, q.start0, q.len0, ids0, ev.junc)) { ev.bad = true; return; }
    if (q.tid1->empty()) return;
    if (!readTranscripts(g, *q.tid1, q.tstart1, q.start1, q.len1, ids1, ev.junc)) { ev.bad = true; return; }
    std::string geneId;
    for (auto &x : ids0) {
        if (!ids1.count(x)) continue;
        auto tp = g->transcripts.find(x);
        if (tp == g->transcripts.end()) { ev.bad = true; return; }
        ev.tr.push_back(const_cast<GtfTranscript *>(&tp->second));
        geneId = tp->second.geneId;
    }
    if (ev.tr.empty()) return;
    auto ge = g->genes.find(geneId);
    if (ge == g->genes.end()) { ev.bad = true; return; }
    ev.gene = const_cast<GtfGene *>(&ge->second);
}

static void applyEvent(const GtfPairEvent &ev) {
    for (GtfFeature *f : ev.junc) f->readCount++;
    for (GtfTranscript *t : ev.tr) t->readCount += 1.f / (float)ev.tr.size();
    if (ev.gene) ev.gene->readCount++;
}

// GTFReader::IncrementReadCount (pair form) for one pair
bool gtfCountPair(snapgpu_gtf_t *g, const std::string &tid0, uint32_t tstart0, uint32_t start0, uint32_t len0,
                  const std::string &tid1, uint32_t tstart1, uint32_t start1, uint32_t len1) {
    GtfPairEvent ev;
    pairEvent(g, GtfPairQuery{&tid0, tstart0, start0, len0, &tid1, tstart1, start1, len1}, ev);
    if (ev.bad) return false;
    applyEvent(ev);
    return true;
}

// The same for a batch of pairs in input order: the interval queries run on host threads (read
// only), the counter updates afterwards in pair order, so the float transcript counts add up in
// the reference's order.  Returns the index of the first pair naming an unknown transcript or
// gene, with no counter touched (every event is checked before any is applied), or -1.
int64_t gtfCountPairs(snapgpu_gtf_t *g, const std::vector<GtfPairQuery> &q) {
    const uint64_t n = q.size();
    std::vector<GtfPairEvent> ev(n);
    const unsigned nt = n < 4096 ? 1u : hostThreads(16);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; i++) pairEvent(g, q[i], ev[i]);
        });
    for (auto &x : th) x.join();
    for (uint64_t i = 0; i < n; i++)
        if (ev[i].bad) return (int64_t)i;
    for (uint64_t i = 0; i < n; i++) applyEvent(ev[i]);
    return -1;
}

}  // namespace snapgpu

extern "C" {

int snapgpu_gtf_reset_counts(snapgpu_gtf_t *g) {
    if (!g) return SNAPGPU_EINVAL;
    for (auto &f : g->features) f.second.readCount = 0;
    for (auto &t : g->transcripts) t.second.readCount = 0.f;
    for (auto &ge : g->genes) ge.second.readCount = 0;
    return SNAPGPU_OK;
}

// ostream << double with the default format (precision 6, %g)
static std::string fmtG(double v) {
    char b[64];
    snprintf(b, sizeof(b), "%g", v);
    return b;
}

int snapgpu_gtf_write_counts(const snapgpu_gtf_t *g, const char *prefix) {
    if (!g || !prefix) return SNAPGPU_EINVAL;
    const std::string p = prefix;
    std::string tid, tname, gid, gname, jid;
    for (auto &t : g->transcripts) {   // GTFTranscript::WriteReadCountID / Name: round(float)
        const std::string c = fmtG(::round((double)t.second.readCount));
        tid += t.first + '\t' + c + '\n';
        tname += t.second.transcriptName + '\t' + c + '\n';
    }
    std::map<std::string, uint32_t> byName;
    for (auto &ge : g->genes) {
        gid += ge.first + '\t' + std::to_string(ge.second.readCount) + '\n';
        // GTFGene::WriteJunctionCountID (:916-924): count / (gene reads / 1000 + 1), rounded
        const float expression = (float)(((float)ge.second.readCount / 1000.0) + 1);
        for (auto &in : ge.second.introns) {
            const GtfFeature *f = in.second;
            jid += ge.first + ":" + f->chr + ':' + u32s(f->start) + "-" + u32s(f->end) + '\t' +
                   fmtG(::round((double)((float)f->readCount / expression))) + '\n';
        }
        auto it = byName.find(ge.second.geneName);
        if (it == byName.end()) byName.insert({ge.second.geneName, ge.second.readCount});
        else it->second += ge.second.readCount;
    }
    for (auto &x : byName) gname += x.first + '\t' + std::to_string(x.second) + '\n';
    const std::pair<const char *, const std::string *> files[] = {
        {".transcript_id.counts.txt", &tid}, {".gene_id.counts.txt", &gid}, {".junction_id.counts.txt", &jid},
        {".transcript_name.counts.txt", &tname}, {".gene_name.counts.txt", &gname}, {".junction_name.counts.txt", nullptr}};
    for (auto &f : files) {
        FILE *o = fopen((p + f.first).c_str(), "w");
        if (!o) { setError("cannot write " + p + f.first); return SNAPGPU_EIO; }
        bool ok = !f.second || fwrite(f.second->data(), 1, f.second->size(), o) == f.second->size();
        if (fclose(o) != 0 || !ok) { setError("write failed: " + p + f.first); return SNAPGPU_EIO; }
    }
    return SNAPGPU_OK;
}

}  // extern "C"

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
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace snapgpu {

struct GtfFeature {
    std::string key, chr, feature, geneId, transcriptId;
    uint32_t start = 0, end = 0;
    int type = 0;   // 1 exon, 2 intron (GTFReader.h:49)
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
    std::string chr, geneId, transcriptId;
    uint32_t start = 0, end = 0;
    std::vector<const GtfFeature *> features;   // exon lines, in file order
    std::vector<const GtfFeature *> exons;      // after Process: exons and introns by start
};

struct Gtf {
    std::map<std::string, GtfFeature> features;          // feature_map (keys stable: pointers stay valid)
    std::map<std::string, GtfTranscript> transcripts;    // transcript_map
    std::map<std::string, std::set<std::string>> genes;  // gene_id -> transcript ids
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
                    t.start = f.start; t.end = f.end;
                    t.features.push_back(fe);
                    g->transcripts.insert({f.transcriptId, t});
                } else {
                    tp->second.features.push_back(fe);
                    tp->second.start = std::min(tp->second.start, f.start);   // UpdateBoundaries
                    tp->second.end = std::max(tp->second.end, f.end);
                }
                g->genes[f.geneId].insert(f.transcriptId);
            }
        }
        std::getline(in, line, '\n');
    }
    // genes in gene_id order, each gene's transcripts in id order: GTFTranscript::Process
    for (auto &gene : g->genes)
        for (auto &tid : gene.second) {
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
                    t.exons.push_back(&ip->second);
                }
                t.exons.push_back(cur);
                prev = cur;
            }
        }
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

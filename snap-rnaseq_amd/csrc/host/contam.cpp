// contam.cpp -- the contamination database's counts (`-ct`, SURVEY.md 8(f) f1/f4 remainder):
// ContaminationFilter (SNAPLib/ContaminationFilter.cpp:22-112).  The product paths
// (single.cpp, rna_paired.cpp) run the contamination aligners on the GPU and add each aligned
// contaminant location here; Write reproduces ContaminationFilter::Write's file.
#include "internal.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace snapgpu;

struct snapgpu_contaminants {
    const Genome *genome = nullptr;           // the contamination index's genome
    std::map<std::string, unsigned> counts;   // contamination_count, keyed by contig name
    mutable std::mutex mu;
};

namespace {

// Contaminant (ContaminationFilter.h:35-56): ordered by count only
struct Contaminant {
    std::string rname;
    unsigned count;
    bool operator<(const Contaminant &r) const { return count < r.count; }
};

// ContaminationFilter::Write's text: the counts in name order, std::sort over reverse iterators
// (descending by count; ties in the order that sort leaves them, as the reference's own call)
std::string formatCounts(const snapgpu_contaminants *c) {
    std::vector<Contaminant> temp;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        for (auto &kv : c->counts) temp.push_back(Contaminant{kv.first, kv.second});
    }
    std::sort(temp.rbegin(), temp.rend());
    std::string out;
    for (auto &t : temp) {
        out += t.rname;
        out += '\t';
        out += std::to_string(t.count);
        out += '\n';
    }
    return out;
}

}  // namespace

namespace snapgpu {

// Every location's contig, or -1 when the location lies before the first contig (the reference
// dereferences the NULL piece there); -2 for a location that counts nothing ("*", or position 0).
static int contigOf(const Genome &g, uint32_t location) {
    if (location == 0xffffffffu) return -2;   // rname "*", pos 0: nothing counted
    const auto &po = g.pieceOffsets;
    int lo = 0, hi = (int)po.size() - 1, p = -1;
    while (lo <= hi) {   // Genome::getPieceAtLocation (Genome.cpp:356-374)
        const int mid = (lo + hi) / 2;
        if (po[mid] <= location && (mid == (int)po.size() - 1 || po[mid + 1] > location)) { p = mid; break; }
        else if (po[mid] <= location) lo = mid + 1;
        else hi = mid - 1;
    }
    if (p < 0) return -1;
    return location - po[p] + 1 == 0 ? -2 : p;
}

// AddAlignment of every location, all or nothing: the locations are resolved first, and a call
// with one unresolvable location changes no count (the product paths add a call's contaminants
// only after every step that can fail has passed).  apply = false only checks.
int contaminantsAddAll(snapgpu_contaminants_t *c, const std::vector<uint32_t> &locations, bool apply) {
    const Genome &g = *c->genome;
    std::vector<int> piece(locations.size());
    for (size_t i = 0; i < locations.size(); i++)
        if ((piece[i] = contigOf(g, locations[i])) == -1) {
            setError("contaminants_add: location before the first contig");
            return SNAPGPU_EINVAL;
        }
    if (!apply) return SNAPGPU_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    for (int p : piece)
        if (p >= 0) c->counts[g.pieceNames[p]]++;
    return SNAPGPU_OK;
}

}  // namespace snapgpu

extern "C" {

snapgpu_contaminants_t *snapgpu_contaminants_create(const snapgpu_index_t *contamination) {
    if (!contamination || !contamination->genome) { setError("contaminants_create: no index"); return nullptr; }
    auto *c = new snapgpu_contaminants();
    c->genome = contamination->genome;
    return c;
}

void snapgpu_contaminants_free(snapgpu_contaminants_t *c) { delete c; }

// ContaminationFilter::AddAlignment (ContaminationFilter.cpp:42-77): the contig of the location
// (Genome::getPieceAtLocation) and 1-based position; counted when the position is not 0
int snapgpu_contaminants_add(snapgpu_contaminants_t *c, uint32_t location) {
    if (!c) return SNAPGPU_EINVAL;
    return snapgpu::contaminantsAddAll(c, std::vector<uint32_t>{location});
}

int snapgpu_contaminants_format(const snapgpu_contaminants_t *c, char *out, uint64_t cap, uint64_t *used) {
    if (!c || !used) return SNAPGPU_EINVAL;
    const std::string s = formatCounts(c);
    *used = s.size();
    if (!out) return SNAPGPU_OK;
    if (cap < s.size()) return SNAPGPU_EINVAL;
    memcpy(out, s.data(), s.size());
    return SNAPGPU_OK;
}

int snapgpu_contaminants_write(const snapgpu_contaminants_t *c, const char *outputFileTemplate) {
    if (!c) return SNAPGPU_EINVAL;
    // ContaminationFilter::ContaminationFilter (:25-35): prefix = the template up to its last '.'
    std::string prefix = "default";
    if (outputFileTemplate) {
        prefix = outputFileTemplate;
        const size_t pos = prefix.rfind('.');
        if (pos != std::string::npos) prefix = prefix.substr(0, pos);
    }
    const std::string path = prefix + ".contaminants.txt", s = formatCounts(c);
    FILE *f = fopen(path.c_str(), "w");
    if (!f) { setError("cannot write " + path); return SNAPGPU_EIO; }
    const bool ok = fwrite(s.data(), 1, s.size(), f) == s.size();
    if (fclose(f) != 0 || !ok) { setError("write failed: " + path); return SNAPGPU_EIO; }
    return SNAPGPU_OK;
}

}  // extern "C"

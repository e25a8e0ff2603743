// sam.cpp -- SAM lines of single-end genome alignments, host side.
//
// SAMFormat::writeRead (SNAPLib/SAM.cpp:1007-1155) with getSAMData
// (SAM.cpp:804-975) for a read without mate, without transcriptome and without
// clipping: the per-read LV-with-CIGAR work comes from the GPU
// (snapgpu_cigar_resident / snapgpu_cigar_batch); this file only prints.  Lines
// are formatted in parallel chunks and concatenated in read order.
#include "internal.h"

#include <algorithm>
#include <cstdio>
#include <map>
#include <string>
#include <cstring>
#include <thread>
#include <vector>

using namespace snapgpu;

namespace {

const int SAM_MULTI_SEGMENT = 0x001;        // SAM.h:38-46
const int SAM_ALL_ALIGNED = 0x002;
const int SAM_UNMAPPED = 0x004;
const int SAM_NEXT_UNMAPPED = 0x008;
const int SAM_REVERSE_COMPLEMENT = 0x010;
const int SAM_NEXT_REVERSED = 0x020;
const int SAM_FIRST_SEGMENT = 0x040;
const int SAM_LAST_SEGMENT = 0x080;

inline char upperCase(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 0x20) : c; }   // Tables.cpp:74-80
inline char complement(char c) {                                                         // Tables.cpp:22-30
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        case 'N': return 'N';
        case 'n': return 'n';
        default: return 0;
    }
}

// Genome::getPieceAtLocation (Genome.cpp:357-374)
// upperCase and COMPLEMENT[upperCase(c)] as 256-entry tables (SEQ of forward / RC records)
struct SeqTables {
    char up[256], rcUp[256];
    SeqTables() {
        for (int c = 0; c < 256; c++) {
            up[c] = upperCase((char)c);
            rcUp[c] = complement(upperCase((char)c));
        }
    }
};
const SeqTables kSeq;
const char *const kUpper = kSeq.up;
const char *const kRcUpper = kSeq.rcUp;

int pieceAt(const Genome &g, uint32_t loc) {
    int lo = 0, hi = (int)g.pieceOffsets.size() - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (g.pieceOffsets[mid] <= loc && (mid == (int)g.pieceOffsets.size() - 1 || g.pieceOffsets[mid + 1] > loc))
            return mid;
        else if (g.pieceOffsets[mid] <= loc) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// decimal without snprintf (the lines are written at millions per second)
inline void appendUint(std::string &o, uint64_t v) {
    char b[24];
    int k = 0;
    do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) o += b[--k];
}
inline void appendInt(std::string &o, int64_t v) {
    if (v < 0) { o += '-'; appendUint(o, (uint64_t)(-v)); }
    else appendUint(o, (uint64_t)v);
}

struct Job {
    const Index *idx;
    const snapgpu_reads_t *reads;
    const char *ids;
    const uint64_t *idOffsets;
    const uint32_t *idLengths;
    const snapgpu_result_t *res;
    const int32_t *ed;
    const uint32_t *nOps;
    const uint32_t *ops;
    const char *rg;
    const uint32_t *front;       // Read::getFrontClippedLength per read, or null (unclipped)
    const uint32_t *unclipped;   // Read::getUnclippedLength per read, or null
};

void formatOne(const Job &J, uint64_t i, std::string &o) {
    const snapgpu_result_t &r = J.res[i];
    SamLine L;
    L.id = J.ids + J.idOffsets[i];
    L.idLen = J.idLengths[i];
    // SEQ / QUAL are the unclipped read (getSAMData, SAM.cpp:866-883); offsets/lengths are the
    // clipped read the aligner saw (Read::clip, Read.h:357-404)
    L.front = J.front ? J.front[i] : 0u;
    L.clippedLen = J.reads->lengths[i];
    L.fullLen = J.unclipped ? J.unclipped[i] : L.clippedLen;
    L.bases = J.reads->bases + J.reads->offsets[i] - L.front;
    L.quals = J.reads->quals + J.reads->offsets[i] - L.front;
    L.result = r.result;
    L.loc = r.location;
    L.dir = r.direction;
    L.mapq = r.mapq;
    L.ed = J.ed[i];
    L.ops = J.ops + i * SNAPGPU_CIGAR_MAX_OPS;
    L.nOps = J.nOps[i];
    L.rg = J.rg;
    samAppendLine(o, *J.idx->genome, L);
}

}  // namespace

namespace snapgpu {

// One SAMFormat::writeRead line (SAM.cpp:1007-1155 with getSAMData, :804-975) for a read
// without mate.
void samAppendLine(std::string &o, const Genome &g, const SamLine &L) {
    static const char kOp[] = "MIDNSHP=X";
    // getSAMData: NotFound -> unmapped, unmapped -> forward
    uint32_t loc = L.loc;
    if (L.result == SNAPGPU_NOT_FOUND) loc = kInvalidLocation;
    const int rc = loc != kInvalidLocation && L.dir == SNAPGPU_RC;
    int flags = 0, mapq = 0;
    const char *pieceName = "*";
    int pieceIdx = -1;
    uint32_t pos = 0;
    if (loc != kInvalidLocation) {
        if (rc) flags |= SAM_REVERSE_COMPLEMENT;
        int p = pieceAt(g, loc);
        if (p >= 0) {
            pieceName = g.pieceNames[p].c_str();
            pieceIdx = p;
            pos = loc - g.pieceOffsets[p] + 1;
        }
        mapq = std::max(0, std::min(70, L.mapq));
    } else {
        flags |= SAM_UNMAPPED;
    }
    // mate fields (SAM.cpp:914-973): RNEXT "=" unless both are mapped on different pieces
    // (the reference compares piece-name pointers), TLEN from the clipped-read extents
    const char *mateName = "*";
    uint32_t matePos = 0;
    int64_t tlen = 0;
    if (L.hasMate) {
        flags |= SAM_MULTI_SEGMENT | (L.firstInPair ? SAM_FIRST_SEGMENT : SAM_LAST_SEGMENT);
        int mateIdx = -1;
        if (L.mateLoc != kInvalidLocation) {
            const int mp = pieceAt(g, L.mateLoc);
            if (mp >= 0) {
                mateName = g.pieceNames[mp].c_str();
                mateIdx = mp;
                matePos = L.mateLoc - g.pieceOffsets[mp] + 1;
            }
            if (L.mateDir == SNAPGPU_RC) flags |= SAM_NEXT_REVERSED;
            if (loc == kInvalidLocation) {   // the unmapped end takes the mate's RNAME / POS
                pieceName = mateName;
                pieceIdx = -2;               // a different pointer from mateName below
                mateName = "=";
                pos = matePos;
            }
        } else {
            flags |= SAM_NEXT_UNMAPPED;
            mateName = "=";
            matePos = pos;
        }
        if (loc != kInvalidLocation && L.mateLoc != kInvalidLocation) {
            flags |= SAM_ALL_ALIGNED;
            const uint32_t back = L.fullLen - L.clippedLen - L.front;
            const uint32_t before = rc ? back : L.front, after = rc ? L.front : back;
            const int64_t myStart = (int64_t)(uint32_t)(loc - before);
            const int64_t myEnd = (int64_t)(uint32_t)(loc + L.clippedLen + after);
            const int64_t mBefore = L.mateFront, mAfter = (int64_t)L.mateFullLen - L.mateClippedLen - L.mateFront;
            const int64_t mateStart = (int64_t)L.mateLoc - (L.mateDir == SNAPGPU_RC ? mAfter : mBefore);
            const int64_t mateEnd = (int64_t)L.mateLoc + L.mateClippedLen + (L.mateDir == SNAPGPU_FORWARD ? mAfter : mBefore);
            if (pieceIdx >= 0 && pieceIdx == mateIdx) tlen = myStart < mateStart ? mateEnd - myStart : -(myEnd - mateStart);
        }
        if (pieceIdx >= 0 && pieceIdx == mateIdx) mateName = "=";
    }
    // The line is written into a thread-local scratch buffer with raw stores and appended once
    // (one append per line instead of one per field or digit).
    uint32_t qlen = L.qnameLen ? L.qnameLen : L.idLen;
    if (const void *sp = memchr(L.id, ' ', qlen)) qlen = (uint32_t)((const char *)sp - L.id);
    const size_t pieceLen = strlen(pieceName), mateLen = strlen(mateName), rgLen = L.rg ? strlen(L.rg) : 0;
    const uint32_t len = L.fullLen;
    const uint32_t n = len < 1024 ? len : 1024;
    const size_t bound = qlen + pieceLen + mateLen + rgLen + (L.cigar ? L.cigar->size() : 0) + 12 * (size_t)L.nOps +
                         2 * (size_t)n + 256;
    thread_local std::vector<char> scratch;
    if (scratch.size() < bound) scratch.resize(bound * 2);
    char *w = scratch.data();
    auto put = [&w](const char *p, size_t k) { memcpy(w, p, k); w += k; };
    auto putU = [&w](uint64_t v) {
        char b[24];
        int k = 0;
        do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (k) *w++ = b[--k];
    };
    auto putI = [&](int64_t v) {
        if (v < 0) { *w++ = '-'; putU((uint64_t)(-v)); }
        else putU((uint64_t)v);
    };
    put(L.id, qlen);
    *w++ = '\t';
    putI(flags);
    *w++ = '\t';
    put(pieceName, pieceLen);
    *w++ = '\t';
    putU(pos);
    *w++ = '\t';
    putI(mapq);
    *w++ = '\t';
    // CIGAR: computed at writeRead's own location (even for NotFound) -- SAM.cpp:1041-1066
    const int32_t ed = L.loc != kInvalidLocation ? L.ed : -1;
    if (L.loc != kInvalidLocation && L.cigar) {
        put(L.cigar->data(), L.cigar->size());   // transcriptome record: insertSpliceJunctions output (may be empty)
    } else if (L.loc != kInvalidLocation && ed >= 0) {
        // soft clips around the CIGAR (computeCigarString, SAM.cpp:1212-1226); for RC the
        // clipped-before count is the read's back clip (getSAMData, SAM.cpp:870-872)
        const uint32_t back = L.fullLen - L.clippedLen - L.front;
        const uint32_t before = rc ? back : L.front, after = rc ? L.front : back;
        if (before) { putU(before); *w++ = 'S'; }
        for (uint32_t k = 0; k < L.nOps; k++) {
            putU(L.ops[k] >> 4);
            *w++ = kOp[L.ops[k] & 15];
        }
        if (after) { putU(after); *w++ = 'S'; }
    } else {
        *w++ = '*';
    }
    *w++ = '\t';
    put(mateName, mateLen);
    *w++ = '\t';
    putU(matePos);
    *w++ = '\t';
    putI(tlen);
    *w++ = '\t';
    // SEQ / QUAL are printed with "%.*s" (SAM.cpp:1122-1136): a NUL byte ends them early
    // (COMPLEMENT[] of a non-ACGTN base is 0; a quality string shorter than the read)
    const unsigned char *B = reinterpret_cast<const unsigned char *>(L.bases);
    if (rc) {
        for (uint32_t k = 0; k < n; k++) {
            const char c = kRcUpper[B[len - 1 - k]];
            if (!c) break;
            *w++ = c;
        }
        *w++ = '\t';
        for (uint32_t k = 0; k < n && L.quals[len - 1 - k]; k++) *w++ = L.quals[len - 1 - k];
    } else {
        for (uint32_t k = 0; k < n; k++) {
            const char c = kUpper[B[k]];
            if (!c) break;
            *w++ = c;
        }
        *w++ = '\t';
        for (uint32_t k = 0; k < n && L.quals[k]; k++) *w++ = L.quals[k];
    }
    if (L.rg) {
        put("\tRG:Z:", 6);
        put(L.rg, rgLen);
    }
    put("\tPG:Z:SNAP\tNM:i:", 16);
    putI(ed);
    *w++ = '\n';
    o.append(scratch.data(), (size_t)(w - scratch.data()));
}

}  // namespace snapgpu

namespace {
}  // namespace

extern "C" int snapgpu_sam_format_clipped(const snapgpu_index_t *idx, const snapgpu_reads_t *reads, const char *ids,
                                          const uint64_t *idOffsets, const uint32_t *idLengths,
                                          const snapgpu_result_t *results, const int32_t *editDistance,
                                          const uint32_t *nOps, const uint32_t *ops, const char *readGroup,
                                          const uint32_t *frontClipped, const uint32_t *unclippedLength, char *out,
                                          uint64_t cap, uint64_t *used) {
    if (!idx || !reads || !ids || !idOffsets || !idLengths || !results || !editDistance || !nOps || !ops || !used) {
        setError("sam_format: null argument");
        return SNAPGPU_EINVAL;
    }
    for (uint64_t i = 0; i < reads->n; i++)
        if (nOps[i] > SNAPGPU_CIGAR_MAX_OPS || (unclippedLength ? unclippedLength[i] : reads->lengths[i]) > 1024 ||
            (unclippedLength && (!frontClipped || unclippedLength[i] < reads->lengths[i] + frontClipped[i] ||
                                 reads->offsets[i] < frontClipped[i]))) {   // the reference writer: <= 500
            setError("sam_format: nOps > SNAPGPU_CIGAR_MAX_OPS, read longer than 1024 bases or bad clip arrays");
            return SNAPGPU_EINVAL;
        }
    if (reads->frontClipped && unclippedLength)   // caller arrays must describe the batch's clip state
        for (uint64_t i = 0; i < reads->n; i++)
            if (frontClipped[i] != reads->frontClipped[i] || unclippedLength[i] != reads->unclippedLength[i]) {
                setError("sam_format: clip arrays differ from the batch's clip state (snapgpu_reads_clip)");
                return SNAPGPU_EINVAL;
            }
    if (!unclippedLength && reads->frontClipped) {   // the batch knows its own clips
        frontClipped = reads->frontClipped;
        unclippedLength = reads->unclippedLength;
    }
    Job J{idx, reads, ids, idOffsets, idLengths, results, editDistance, nOps, ops, readGroup,
          unclippedLength ? frontClipped : nullptr, unclippedLength};
    const uint64_t n = reads->n;
    unsigned nt = hostThreads(16);
    if (n < 4096) nt = 1;
    std::vector<std::string> parts(nt);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
            // a local string, swapped in at the end: the parts' headers share cache lines, and
            // appending through them bounced those lines between the threads
            std::string o;
            o.reserve((b - a) * 320);
            for (uint64_t i = a; i < b; i++) formatOne(J, i, o);
            parts[t].swap(o);
        });
    for (auto &x : th) x.join();
    uint64_t total = 0;
    for (auto &p : parts) total += p.size();
    *used = total;
    if (total > cap || (!out && total)) {
        setError("sam_format: output buffer too small");
        return SNAPGPU_EINVAL;
    }
    // each thread copies its own part (the first touch of the caller's pages and ~300 MB of copy
    // per 1M lines run in parallel, not on one thread after the join)
    std::vector<uint64_t> at(nt + 1, 0);
    for (unsigned t = 0; t < nt; t++) at[t + 1] = at[t] + parts[t].size();
    th.clear();
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            memcpy(out + at[t], parts[t].data(), parts[t].size());
            std::string().swap(parts[t]);
        });
    for (auto &x : th) x.join();
    return SNAPGPU_OK;
}

extern "C" int snapgpu_sam_format(const snapgpu_index_t *idx, const snapgpu_reads_t *reads, const char *ids,
                                  const uint64_t *idOffsets, const uint32_t *idLengths,
                                  const snapgpu_result_t *results, const int32_t *editDistance, const uint32_t *nOps,
                                  const uint32_t *ops, const char *readGroup, char *out, uint64_t cap,
                                  uint64_t *used) {
    return snapgpu_sam_format_clipped(idx, reads, ids, idOffsets, idLengths, results, editDistance, nOps, ops,
                                      readGroup, nullptr, nullptr, out, cap, used);
}

// Read::clip (Read.h:357-404) on every read of a batch, in place: offsets/lengths become the
// clipped read; frontClipped / unclippedLength receive what the SAM writer needs (and are kept
// in the batch).  As Read::clip: a no-op when the batch is already in that state, otherwise the
// read is restored to its unclipped extent first, so clip(3) twice or clip(3) then clip(0) give
// the reference's reads.  Refused once the batch has been uploaded (the device copy would keep
// the old extents while the SAM writer prints the new clips).
extern "C" int snapgpu_reads_clip(snapgpu_reads_t *r, int clipping, uint32_t *frontClipped,
                                  uint32_t *unclippedLength) {
    if (!r || clipping < 0 || clipping > 3) {
        setError("reads_clip: bad argument");
        return SNAPGPU_EINVAL;
    }
    const bool same = r->frontClipped ? clipping == r->clipping : clipping == 0;
    if (r->nUploads && !same) {   // Read::clip returns early when the state is unchanged (Read.h:361-363)
        setError("reads_clip: the batch was already uploaded to a device; clip before uploading");
        return SNAPGPU_EINVAL;
    }
    if (!r->frontClipped) {   // first clip: remember the unclipped extents
        r->frontClipped = new uint32_t[r->n + 1]();
        r->unclippedLength = new uint32_t[r->n + 1]();
        for (uint64_t i = 0; i < r->n; i++) r->unclippedLength[i] = r->lengths[i];
        r->clipping = 0;
    }
    if (clipping != r->clipping) {
        for (uint64_t i = 0; i < r->n; i++) {
            // revert to unclipped (Read.h:369-372)
            r->offsets[i] -= r->frontClipped[i];
            const uint32_t full = r->unclippedLength[i];
            const char *q = r->quals + r->offsets[i];
            uint32_t len = full, front = 0;
            if (clipping == 2 || clipping == 3)   // ClipBack / ClipFrontAndBack
                while (len > 0 && q[len - 1] == '#') len--;
            if (clipping == 1 || clipping == 3)   // ClipFront / ClipFrontAndBack
                while (front < len && q[front] == '#') front++;
            if (len - front < 50) { len = full; front = 0; }   // "just use all of it" (Read.h:393-397)
            else len -= front;
            r->frontClipped[i] = front;
            r->offsets[i] += front;
            r->lengths[i] = len;
        }
        r->clipping = clipping;
    }
    if (frontClipped) memcpy(frontClipped, r->frontClipped, r->n * sizeof(uint32_t));
    if (unclippedLength) memcpy(unclippedLength, r->unclippedLength, r->n * sizeof(uint32_t));
    return SNAPGPU_OK;
}

// SAMFormat::writeHeader (SAM.cpp:700-800) for an input without its own header (FASTQ):
// @HD, the read-group line, @PG, then one @SQ per genome piece with LN = piece span - 500
// (the reference subtracts a fixed 500, whatever the padding; unsigned arithmetic kept).
extern "C" int snapgpu_sam_header(const snapgpu_index_t *idx, int sorted, const char *commandLine,
                                  const char *version, const char *rgLine, char *out, uint64_t cap, uint64_t *used) {
    if (!idx || !commandLine || !version || !used) {
        setError("sam_header: null argument");
        return SNAPGPU_EINVAL;
    }
    const Genome &g = *idx->genome;
    std::string o = "@HD\tVN:1.4\tSO:";
    o += sorted ? "coordinate" : "unsorted";
    o += '\n';
    o += rgLine ? rgLine : "@RG\tID:FASTQ\tSM:sample";
    o += "\n@PG\tID:SNAP\tPN:SNAP\tCL:";
    o += commandLine;
    o += "\tVN:";
    o += version;
    o += '\n';
    const size_t np = g.pieceOffsets.size();
    for (size_t i = 0; i < np; i++) {
        const uint32_t start = g.pieceOffsets[i], end = i + 1 < np ? g.pieceOffsets[i + 1] : g.nBases;
        o += "@SQ\tSN:";
        o += g.pieceNames[i];
        o += "\tLN:";
        appendUint(o, (uint32_t)((end - start) - 500u));
        o += '\n';
    }
    *used = o.size();
    if (o.size() > cap || !out) {
        setError("sam_header: output buffer too small");
        return SNAPGPU_EINVAL;
    }
    memcpy(out, o.data(), o.size());
    return SNAPGPU_OK;
}

namespace snapgpu {

// SAMFormat::getSortInfo's location of one record (SAM.cpp:639-685 with SAMReader::parsePieceName
// and parseLocation, :408-468): POS empty or '*' -> the mate's RNEXT/PNEXT (UINT32_MAX when PNEXT is
// '*' too), else RNAME/POS; an RNAME that is '*' gives InvalidGenomeLocation, a name the genome does
// not know (RNEXT "=") offset 0; location = piece offset + POS - 1.
static uint32_t samSortKey(const std::map<std::string, uint32_t> &pieces, const char *line, size_t len) {
    const char *f[9];
    size_t fl[9];
    size_t k = 0, start = 0;
    for (size_t i = 0; i <= len && k < 9; i++)
        if (i == len || line[i] == '\t') { f[k] = line + start; fl[k] = i - start; k++; start = i + 1; }
    for (; k < 9; k++) { f[k] = line + len; fl[k] = 0; }
    auto loc = [&](int rf, int pf) -> uint32_t {
        if (fl[rf] == 0 || fl[pf] == 0 || f[rf][0] == '*' || f[pf][0] == '*') return 0xffffffffu;
        const auto it = pieces.find(std::string(f[rf], fl[rf]));
        const uint32_t off = it == pieces.end() ? 0u : it->second;
        uint32_t pos = 0;
        for (size_t i = 0; i < fl[pf] && f[pf][i] >= '0' && f[pf][i] <= '9'; i++) pos = pos * 10 + (uint32_t)(f[pf][i] - '0');
        return off + pos - 1;
    };
    if (fl[3] == 0 || f[3][0] == '*') return (fl[7] == 0 || f[7][0] == '*') ? 0xffffffffu : loc(6, 7);
    return loc(2, 3);
}

std::string samSortRecords(const Genome &g, const std::vector<std::string> &parts) {
    std::map<std::string, uint32_t> pieces;
    for (size_t i = 0; i < g.pieceNames.size(); i++) pieces.emplace(g.pieceNames[i], g.pieceOffsets[i]);
    struct Rec { uint32_t key; const char *p; size_t n; };
    std::vector<Rec> recs;
    size_t total = 0;
    for (const auto &s : parts) {
        total += s.size();
        size_t b = 0;
        while (b < s.size()) {
            size_t e = s.find('\n', b);
            e = e == std::string::npos ? s.size() : e + 1;
            recs.push_back(Rec{samSortKey(pieces, s.data() + b, e - b - (s[e - 1] == '\n')), s.data() + b, e - b});
            b = e;
        }
    }
    std::stable_sort(recs.begin(), recs.end(), [](const Rec &a, const Rec &b) { return a.key < b.key; });
    std::string out;
    out.reserve(total);
    for (const auto &r : recs) out.append(r.p, r.n);
    return out;
}

}  // namespace snapgpu

extern "C" int snapgpu_sam_sort_records(const snapgpu_index_t *idx, const char *in, uint64_t n, char *out, uint64_t cap,
                                        uint64_t *used) {
    if (!idx || !idx->genome || (!in && n) || !used) return SNAPGPU_EINVAL;
    if (n && in[n - 1] != '\n') {   // a last record without its newline would be joined to the next
        setError("sam_sort_records: the records must end with a newline");
        return SNAPGPU_EINVAL;
    }
    *used = n;
    if (!out) return SNAPGPU_OK;
    if (cap < n) return SNAPGPU_EINVAL;
    const std::string sorted = samSortRecords(*idx->genome, std::vector<std::string>{std::string(in, n)});
    memcpy(out, sorted.data(), sorted.size());
    return SNAPGPU_OK;
}

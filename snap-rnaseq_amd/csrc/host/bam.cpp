// bam.cpp -- BAM output of the single-end and RNA paired product paths:
// BAMFormat::writeHeader / writeRead (SNAPLib/Bam.cpp:542-790) over the same per-record fields
// the SAM writer prints (getSAMData, SAM.cpp:804-975), and a BGZF stream (the reference's
// GzipWriterFilter with 64 KB blocks, DataWriterSupplier::gzip(true, 0x10000, ...)).
//
// Kept from the reference: the QNAME is the whole read id (qnameLen, not cut at the first space as
// the SAM text is); SEQ and QUAL cover the whole unclipped read (no "%.*s" NUL stop); an unmapped
// record carries no CIGAR, and its NM is the previous record's (writeRead's editDistance is only
// set when a CIGAR is computed -- the caller passes that value in); bin = reg2bin of the record's
// reference span, (-1, 0) for an unmapped read without mate.
#include "internal.h"

#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>

namespace snapgpu {

namespace {

const int SAM_MULTI_SEGMENT = 0x001;       // SAM.h:38-46
const int SAM_ALL_ALIGNED = 0x002;
const int SAM_UNMAPPED = 0x004;
const int SAM_NEXT_UNMAPPED = 0x008;
const int SAM_REVERSE_COMPLEMENT = 0x010;
const int SAM_NEXT_REVERSED = 0x020;
const int SAM_FIRST_SEGMENT = 0x040;
const int SAM_LAST_SEGMENT = 0x080;

inline char upperCase(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 0x20) : c; }
inline char complementOf(char c) {
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

// BAMAlignment::SeqToCode from CodeToSeq = "=ACMGRSVTWYHKDBN" (Bam.cpp:179, :266-276)
struct SeqCode {
    uint8_t v[256];
    SeqCode() {
        memset(v, 0, sizeof(v));
        const char *c = "=ACMGRSVTWYHKDBN";
        for (int i = 1; i < 16; i++) v[(uint8_t)c[i]] = (uint8_t)i;
    }
};
const SeqCode kSeqCode;
const int kRefBase[16] = {1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};   // CigarCodeToRefBase (Bam.cpp:183)

int reg2bin(int beg, int end) {   // BAMAlignment::reg2bin (Bam.cpp:279-291)
    --end;
    if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
    if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
    if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
    if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
    if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
    return 0;
}

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

template <class T>
void put(std::string &o, T v) { o.append(reinterpret_cast<const char *>(&v), sizeof(T)); }

}  // namespace

// One BAMFormat::writeRead record appended to o (Bam.cpp:596-790): a read without mate, or one end
// of a pair (L.hasMate: getSAMData's mate branch, SAM.cpp:914-973, with piece indices where the SAM
// line has names).  nm: the NM value the reference writes (the record's own edit distance when it
// has a location, else the previous record's).  False if the QNAME is too long for BAM (the
// reference exits, Bam.cpp:723-726).
bool bamAppendRecord(std::string &o, const Genome &g, const SamLine &L, int32_t nm) {
    static const char kOp[] = "MIDNSHP=X";
    uint32_t loc = L.loc;
    if (L.result == SNAPGPU_NOT_FOUND) loc = kInvalidLocation;
    const bool rc = loc != kInvalidLocation && L.dir == SNAPGPU_RC;
    int flags = 0, mapq = 0, pieceIdx = -1;
    uint32_t pos = 0;
    if (loc != kInvalidLocation) {
        if (rc) flags |= SAM_REVERSE_COMPLEMENT;
        const int p = pieceAt(g, loc);
        if (p >= 0) {
            pieceIdx = p;
            pos = loc - g.pieceOffsets[p] + 1;
        }
        mapq = std::max(0, std::min(70, L.mapq));
    } else {
        flags |= SAM_UNMAPPED;
    }
    int mateIdx = -1;
    uint32_t matePos = 0;
    int64_t tlen = 0;
    if (L.hasMate) {
        flags |= SAM_MULTI_SEGMENT | (L.firstInPair ? SAM_FIRST_SEGMENT : SAM_LAST_SEGMENT);
        if (L.mateLoc != kInvalidLocation) {
            const int mp = pieceAt(g, L.mateLoc);
            if (mp >= 0) {
                mateIdx = mp;
                matePos = L.mateLoc - g.pieceOffsets[mp] + 1;
            }
            if (L.mateDir == SNAPGPU_RC) flags |= SAM_NEXT_REVERSED;
            if (loc == kInvalidLocation) {   // the unmapped end takes the mate's RNAME / POS
                pieceIdx = mateIdx;
                pos = matePos;
            }
        } else {                             // the mate is unmapped: it points at this end
            flags |= SAM_NEXT_UNMAPPED;
            mateIdx = pieceIdx;
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
    }
    const uint32_t qlen = L.qnameLen ? L.qnameLen : L.idLen;
    if (qlen > 254) return false;
    // CIGAR ops: computed at writeRead's own location (even for NotFound), soft clips around them
    std::vector<uint32_t> ops;
    if (L.loc != kInvalidLocation && L.cigar) {   // transcriptome record: insertSpliceJunctions output
        uint32_t num = 0;
        for (char c : *L.cigar) {
            if (c >= '0' && c <= '9') { num = num * 10 + (uint32_t)(c - '0'); continue; }
            const char *k = strchr(kOp, c);
            ops.push_back(num << 4 | (uint32_t)(k ? k - kOp : 0));
            num = 0;
        }
    } else if (L.loc != kInvalidLocation && L.ed >= 0) {
        const uint32_t back = L.fullLen - L.clippedLen - L.front;
        const uint32_t before = rc ? back : L.front, after = rc ? L.front : back;
        if (before) ops.push_back(before << 4 | 4u);
        for (uint32_t k = 0; k < L.nOps; k++) ops.push_back(L.ops[k]);
        if (after) ops.push_back(after << 4 | 4u);
    }
    const uint32_t len = L.fullLen;
    int refLength = ops.empty() ? (int)len : 0;
    for (uint32_t op : ops) refLength += kRefBase[op & 15] * (int)(op >> 4);
    // unmapped: at the mate's position, length 1, or at -1 (Bam.cpp:752-756)
    const int bin = L.loc != kInvalidLocation ? reg2bin((int)pos - 1, (int)pos - 1 + refLength)
                  : (L.hasMate && L.mateLoc != kInvalidLocation) ? reg2bin((int)matePos - 1, (int)matePos)
                                                                  : reg2bin(-1, 0);
    const size_t rgLen = L.rg ? strlen(L.rg) : 0;
    const size_t size = 36 + qlen + 1 + 4 * ops.size() + (len + 1) / 2 + len + (L.rg ? 4 + rgLen : 0) + 8 + 7;
    const size_t start = o.size();
    put<int32_t>(o, (int32_t)(size - 4));                // block_size
    put<int32_t>(o, pieceIdx);                           // refID
    put<int32_t>(o, (int32_t)pos - 1);                   // pos
    put<uint8_t>(o, (uint8_t)(qlen + 1));                // l_read_name
    put<uint8_t>(o, (uint8_t)mapq);                      // MAPQ
    put<uint16_t>(o, (uint16_t)bin);
    put<uint16_t>(o, (uint16_t)ops.size());              // n_cigar_op
    put<uint16_t>(o, (uint16_t)flags);
    put<int32_t>(o, (int32_t)len);                       // l_seq
    put<int32_t>(o, mateIdx);                            // next_refID (-1 without mate)
    put<int32_t>(o, (int32_t)matePos - 1);               // next_pos
    put<int32_t>(o, (int32_t)tlen);                      // tlen
    o.append(L.id, qlen);
    o += '\0';
    for (uint32_t op : ops) put<uint32_t>(o, op);
    // SEQ (4-bit codes) and QUAL (phred) of the unclipped read, reverse-complemented for RC
    std::string seq(len, '\0'), qual(len, '\0');
    for (uint32_t i = 0; i < len; i++) {
        if (rc) {
            seq[i] = complementOf(upperCase(L.bases[len - 1 - i]));
            qual[i] = (char)(L.quals[len - 1 - i] - '!');
        } else {
            seq[i] = upperCase(L.bases[i]);
            qual[i] = (char)(L.quals[i] - '!');
        }
    }
    for (uint32_t i = 0; i + 1 < len; i += 2)
        o += (char)(kSeqCode.v[(uint8_t)seq[i]] << 4 | kSeqCode.v[(uint8_t)seq[i + 1]]);
    if (len % 2) o += (char)(kSeqCode.v[(uint8_t)seq[len - 1]] << 4);
    o += qual;
    if (L.rg) {
        o += "RGZ";
        o.append(L.rg, rgLen);
        o += '\0';
    }
    o.append("PGZSNAP\0", 8);
    o += "NMi";
    put<int32_t>(o, nm);
    return o.size() - start == size;   // block_size must describe exactly what was appended
}

// BAMFormat::writeHeader: magic, the SAM header text, one RefSeq per genome piece with
// l_ref = piece length - 500 (Bam.cpp:542-594)
std::string bamHeader(const Genome &g, const std::string &samText) {
    std::string o("BAM\1", 4);
    put<int32_t>(o, (int32_t)samText.size());
    o += samText;
    const size_t np = g.pieceOffsets.size();
    put<int32_t>(o, (int32_t)np);
    for (size_t i = 0; i < np; i++) {
        const std::string &name = g.pieceNames[i];
        put<int32_t>(o, (int32_t)name.size() + 1);
        o += name;
        o += '\0';
        const uint32_t end = i + 1 < np ? g.pieceOffsets[i + 1] : (uint32_t)g.nBases;
        put<int32_t>(o, (int32_t)((end - g.pieceOffsets[i]) - 500u));
    }
    return o;
}

// BGZF: deflate blocks of at most 0xff00 input bytes, each a gzip member with the BC extra field,
// then the empty EOF block.
bool bgzfWrite(FILE *f, const char *data, size_t n, bool eof) {
    static const size_t kIn = 0xff00;
    std::vector<unsigned char> out(compressBound(kIn) + 64);
    for (size_t at = 0; at < n; at += kIn) {
        const size_t m = std::min(kIn, n - at);
        z_stream z;
        memset(&z, 0, sizeof(z));
        if (deflateInit2(&z, Z_DEFAULT_COMPRESSION, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
        z.next_in = (Bytef *)(data + at);
        z.avail_in = (uInt)m;
        z.next_out = out.data() + 18;
        z.avail_out = (uInt)(out.size() - 26);
        const int r = deflate(&z, Z_FINISH);
        const size_t clen = z.total_out;
        deflateEnd(&z);
        if (r != Z_STREAM_END) return false;
        const size_t bsize = 18 + clen + 8;
        const unsigned char hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0,
                                       (unsigned char)((bsize - 1) & 0xff), (unsigned char)((bsize - 1) >> 8)};
        memcpy(out.data(), hdr, 18);
        const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), (const Bytef *)(data + at), (uInt)m);
        memcpy(out.data() + 18 + clen, &crc, 4);
        const uint32_t isize = (uint32_t)m;
        memcpy(out.data() + 22 + clen, &isize, 4);
        if (fwrite(out.data(), 1, bsize, f) != bsize) return false;
    }
    if (eof) {
        static const unsigned char kEof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0,
                                               3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (fwrite(kEof, 1, 28, f) != 28) return false;
    }
    return true;
}

}  // namespace snapgpu

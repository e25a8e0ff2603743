// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on the GPU box).
//
// A small driver linked against the REFERENCE's own SNAPLib objects (built by
// oracle/Makefile.ref from /root/reference) so that the C restatement in
// oracle/snap_oracle.c and the HIP path can be pinned against the real
// BaseAligner / LandauVishkin / GenomeIndex::lookupSeed.
//
// Construction mirrors SNAPLib/SingleAligner.cpp:165-185 (maxReadSize =
// MAX_READ_LENGTH, LV objects owned by the aligner, BigAllocator-backed), and
// the LV tables are initialised as AlignerOptions.cpp:84 does.
//
// Modes:
//   align  <indexDir> <reads.fq> [maxHits maxK numSeeds extraSearchDepth]
//          -> one TSV line per read:
//             i result loc dir score mapq lookups scored popularSkipped pAll_hex pBest_hex
//   alignx <indexDir> <reads.fq> <search.tsv> <maxHitsToGet> [...] -> align columns + multi hits
//   lv     <calls.tsv>   lines: dir k text pattern quals   -> e netIndel prob_hex
//   lookup <indexDir> <seeds.txt>  one seed string per line -> nF nRC sumF sumRC firstF firstRC
//   sam    <indexDir> <reads.fq> [maxHits maxK numSeeds extra [clipping]]
//          -> per read: AlignRead, then the reference's own SAM writer
//             (FileFormat::SAM[useM]->writeRead, SAM.cpp:1007-1155) for useM = 0 and 1:
//             two SAM lines per read
//   samheader <indexDir> <sorted 0|1> <version> [args...]
//          -> SAMFormat::writeHeader (SAM.cpp:700-800) for a FASTQ input (no input header),
//             default read group, command line = args
//   paired <indexDir> <reads0.fq> <reads1.fq> [maxHits maxK numSeeds extra minSpacing maxSpacing maxBigHits]
//          -> per pair: the IntersectingPairedEndAligner result alone, then the
//             ChimericPairedEndAligner result, constructed as PairedAligner.cpp:462-482
//             (paired defaults AlignerOptions.cpp:73-77: maxHits 16000, maxK 15, 8 seeds)
//   cigar  <indexDir> <calls.tsv>  lines: loc dir useM read
//   charseeds <indexDir> <reads.fq> [maxHits maxK numSeeds extra]
//          -> BaseAligner::CharacterizeSeeds (BaseAligner.cpp:206-508) per read with the
//             partial aligner of PairedAligner.cpp:518-527 (maxHits 300, maxK 15, 12 seeds):
//             "i nF nRC F:loc:min:max:count,... RC:loc:min:max:count,..." (std::map order).
//             Needs ref_harness_rna (BaseAligner.cpp at -O0: the function falls off its end,
//             which g++ -O3 compiles into a crash; oracle/Makefile.ref).
//          -> ed cigar   (SAMFormat::computeCigarString, SAM.cpp:1162-1230, restated
//             around the reference's LandauVishkinWithCigar with zeroed slack bytes)
#define private public          // read-only access to BaseAligner's private scoring state
#include "stdafx.h"
#include "BaseAligner.h"
#undef private
#include "GenomeIndex.h"
#include "LandauVishkin.h"
#include "Read.h"
#include "Seed.h"
#include "BigAlloc.h"
#include "FileFormat.h"
#include "Genome.h"
#include "Tables.h"
#include "IntersectingPairedEndAligner.h"
#include "ChimericPairedEndAligner.h"
#include <string>
#include <vector>
#include <fstream>
#include <iostream>
#include <sstream>

static void hexd(double d, char *buf) { sprintf(buf, "%a", d); }

static int mode_align(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "align <indexDir> <reads.fq> [maxHits maxK numSeeds extra]\n"); return 2; }
    unsigned maxHits = argc > 4 ? atoi(argv[4]) : 300;
    unsigned maxK = argc > 5 ? atoi(argv[5]) : 14;
    unsigned numSeeds = argc > 6 ? atoi(argv[6]) : 25;
    unsigned extra = argc > 7 ? atoi(argv[7]) : 2;
    initializeLVProbabilitiesToPhredPlus33();
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) { fprintf(stderr, "cannot load index %s\n", argv[2]); return 1; }
    BigAllocator *al = new BigAllocator(BaseAligner::getBigAllocatorReservation(
        true, maxHits, MAX_READ_LENGTH, idx->getSeedLength(), numSeeds, 0));
    BaseAligner *ba = new (al) BaseAligner(idx, maxHits, maxK, MAX_READ_LENGTH, numSeeds, 0, extra,
                                           NULL, NULL, NULL, al);
    std::ifstream in(argv[3]);
    std::string id, bases, plus, quals;
    unsigned i = 0;
    char b1[64], b2[64];
    while (std::getline(in, id) && std::getline(in, bases) && std::getline(in, plus) && std::getline(in, quals)) {
        std::string b = bases + std::string(16, '\0');   // LV reads up to 8 bytes past the end
        std::string q = quals + std::string(16, '\0');
        Read r;
        r.init(id.c_str() + 1, (unsigned)id.size() - 1, b.c_str(), q.c_str(), (unsigned)bases.size());
        unsigned loc = 0; Direction dir = 0; int score = 0, mapq = 0;
        _int64 l0 = ba->getNHashTableLookups(), s0 = ba->getLocationsScored();
        ba->popularSeedsSkipped = 0;
        ba->probabilityOfAllCandidates = 0; ba->probabilityOfBestCandidate = 0;
        AlignmentResult res = ba->AlignRead(&r, &loc, &dir, &score, &mapq);
        hexd(ba->probabilityOfAllCandidates, b1);
        hexd(ba->probabilityOfBestCandidate, b2);
        printf("%u\t%d\t%u\t%d\t%d\t%d\t%lld\t%lld\t%u\t%s\t%s\n", i, (int)res, loc, dir, score, mapq,
               (long long)(ba->getNHashTableLookups() - l0), (long long)(ba->getLocationsScored() - s0),
               ba->popularSeedsSkipped, b1, b2);
        i++;
    }
    return 0;
}

// alignx <indexDir> <reads.fq> <search.tsv> <maxHitsToGet> [maxHits maxK numSeeds extra]
//   search.tsv: one "radius location direction" line per read.  The richer AlignRead
//   overload (BaseAligner.h:73-86): windowed search + multi-hit export.  Output = the
//   align columns + nFound + "loc:dir:score,..." (or "-").
static int mode_alignx(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "alignx <indexDir> <reads.fq> <search.tsv> <maxHitsToGet> [...]\n"); return 2; }
    int maxGet = atoi(argv[5]);
    unsigned maxHits = argc > 6 ? atoi(argv[6]) : 300;
    unsigned maxK = argc > 7 ? atoi(argv[7]) : 14;
    unsigned numSeeds = argc > 8 ? atoi(argv[8]) : 25;
    unsigned extra = argc > 9 ? atoi(argv[9]) : 2;
    initializeLVProbabilitiesToPhredPlus33();
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) { fprintf(stderr, "cannot load index %s\n", argv[2]); return 1; }
    BigAllocator *al = new BigAllocator(BaseAligner::getBigAllocatorReservation(
        true, maxHits, MAX_READ_LENGTH, idx->getSeedLength(), numSeeds, 0));
    BaseAligner *ba = new (al) BaseAligner(idx, maxHits, maxK, MAX_READ_LENGTH, numSeeds, 0, extra,
                                           NULL, NULL, NULL, al);
    std::ifstream in(argv[3]), sin(argv[4]);
    std::string id, bases, plus, quals;
    unsigned i = 0;
    char b1[64], b2[64];
    std::vector<unsigned> mLoc(maxGet > 0 ? maxGet : 1);
    std::vector<int> mScore(mLoc.size());
    bool *mRC = new bool[mLoc.size()];
    while (std::getline(in, id) && std::getline(in, bases) && std::getline(in, plus) && std::getline(in, quals)) {
        unsigned radius = 0, sloc = 0; int sdir = 0;
        sin >> radius >> sloc >> sdir;
        std::string b = bases + std::string(16, '\0');
        std::string q = quals + std::string(16, '\0');
        Read r;
        r.init(id.c_str() + 1, (unsigned)id.size() - 1, b.c_str(), q.c_str(), (unsigned)bases.size());
        unsigned loc = 0; Direction dir = 0; int score = 0, mapq = 0, found = -7;
        _int64 l0 = ba->getNHashTableLookups(), s0 = ba->getLocationsScored();
        ba->popularSeedsSkipped = 0;
        ba->probabilityOfAllCandidates = 0; ba->probabilityOfBestCandidate = 0;
        AlignmentResult res = ba->AlignRead(&r, &loc, &dir, &score, &mapq, radius, sloc, (Direction)sdir, maxGet,
                                            &found, &mLoc[0], mRC, &mScore[0]);
        hexd(ba->probabilityOfAllCandidates, b1);
        hexd(ba->probabilityOfBestCandidate, b2);
        printf("%u\t%d\t%u\t%d\t%d\t%d\t%lld\t%lld\t%u\t%s\t%s\t%d\t", i, (int)res, loc, dir, score, mapq,
               (long long)(ba->getNHashTableLookups() - l0), (long long)(ba->getLocationsScored() - s0),
               ba->popularSeedsSkipped, b1, b2, found);
        if (found <= 0) printf("-");
        for (int j = 0; j < found; j++) printf("%s%u:%d:%d", j ? "," : "", mLoc[j], (int)mRC[j], mScore[j]);
        printf("\n");
        i++;
    }
    delete[] mRC;
    return 0;
}

static int mode_lv(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "lv <calls.tsv>\n"); return 2; }
    initializeLVProbabilitiesToPhredPlus33();
    LandauVishkin<1> *fwd = new LandauVishkin<1>;
    LandauVishkin<-1> *rev = new LandauVishkin<-1>;
    std::ifstream in(argv[2]);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        int dir, k; std::string text, pattern, quals;
        ss >> dir >> k >> text >> pattern >> quals;
        // Reverse text is walked backwards from its END (LandauVishkin.h:261-263): put
        // the text in a padded buffer and pass a pointer one past its last byte.
        std::string tbuf = std::string(64, 'n') + text + std::string(64, 'n');
        std::string pbuf = pattern + std::string(16, '\0');
        std::string qbuf = quals + std::string(16, '\0');
        double p = 0; int indel = 0; int e;
        if (dir >= 0) e = fwd->computeEditDistance(tbuf.c_str() + 64, (int)text.size(), pbuf.c_str(), qbuf.c_str(),
                                                    (int)pattern.size(), k, &p, 0, &indel);
        else e = rev->computeEditDistance(tbuf.c_str() + 64 + text.size(), (int)text.size(), pbuf.c_str(), qbuf.c_str(),
                                          (int)pattern.size(), k, &p, 0, &indel);
        char b[64]; hexd(p, b);
        printf("%d\t%d\t%s\n", e, indel, b);
    }
    return 0;
}

static int mode_lookup(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "lookup <indexDir> <seeds.txt>\n"); return 2; }
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) return 1;
    std::ifstream in(argv[3]);
    std::string s;
    while (std::getline(in, s)) {
        Seed seed(s.c_str(), idx->getSeedLength());
        unsigned n[2]; const unsigned *h[2];
        idx->lookupSeed(seed, &n[0], &h[0], &n[1], &h[1]);
        unsigned long long sum[2] = {0, 0}; long long first[2] = {-1, -1};
        for (int d = 0; d < 2; d++) {
            for (unsigned j = 0; j < n[d]; j++) sum[d] = sum[d] * 1000003ULL + h[d][j];
            if (n[d]) first[d] = h[d][0];
        }
        printf("%u\t%u\t%llu\t%llu\t%lld\t%lld\n", n[0], n[1], sum[0], sum[1], first[0], first[1]);
    }
    return 0;
}

static int mode_sam(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "sam <indexDir> <reads.fq> [maxHits maxK numSeeds extra]\n"); return 2; }
    unsigned maxHits = argc > 4 ? atoi(argv[4]) : 300;
    unsigned maxK = argc > 5 ? atoi(argv[5]) : 14;
    unsigned numSeeds = argc > 6 ? atoi(argv[6]) : 25;
    unsigned extra = argc > 7 ? atoi(argv[7]) : 2;
    const int clipping = argc > 8 ? atoi(argv[8]) : 0;   // ReadClippingType (Read.h:85), as FASTQ.cpp:250 applies it
    initializeLVProbabilitiesToPhredPlus33();
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) { fprintf(stderr, "cannot load index %s\n", argv[2]); return 1; }
    BigAllocator *al = new BigAllocator(BaseAligner::getBigAllocatorReservation(
        true, maxHits, MAX_READ_LENGTH, idx->getSeedLength(), numSeeds, 0));
    BaseAligner *ba = new (al) BaseAligner(idx, maxHits, maxK, MAX_READ_LENGTH, numSeeds, 0, extra,
                                           NULL, NULL, NULL, al);
    LandauVishkinWithCigar lvc;
    std::ifstream in(argv[3]);
    std::string id, bases, plus, quals;
    std::vector<char> buf(1 << 16);
    while (std::getline(in, id) && std::getline(in, bases) && std::getline(in, plus) && std::getline(in, quals)) {
        std::string b = bases + std::string(16, '\0');
        std::string q = quals + std::string(16, '\0');
        Read r;
        r.init(id.c_str() + 1, (unsigned)id.size() - 1, b.c_str(), q.c_str(), (unsigned)bases.size());
        r.setReadGroup("FASTQ");      // FASTQ.cpp:252 with AlignerOptions.cpp:65's default
        r.clip((ReadClippingType)clipping);
        unsigned loc = 0; Direction dir = 0; int score = 0, mapq = 0;
        AlignmentResult res = ba->AlignRead(&r, &loc, &dir, &score, &mapq);
        for (int useM = 0; useM < 2; useM++) {
            size_t used = 0;
            if (!FileFormat::SAM[useM]->writeRead(idx->getGenome(), NULL, NULL, &lvc, &buf[0], buf.size(), &used, 0,
                                                  &r, res, mapq, loc, dir)) { fprintf(stderr, "writeRead failed\n"); return 1; }
            fwrite(&buf[0], 1, used, stdout);
        }
    }
    return 0;
}


// One line per pair:
//   i  [intersecting: st0 st1 loc0 loc1 dir0 dir1 sc0 sc1 mq0 mq1 nScored]
//      [chimeric:     st0 st1 loc0 loc1 dir0 dir1 sc0 sc1 mq0 mq1 fromAlignTogether alignedAsPair nScored]
// Fields an aligner leaves unwritten keep the pre-state {NotFound, InvalidGenomeLocation, 0, -1, 0}.
static void pairedPre(PairedAlignmentResult &r) {
    memset(&r, 0, sizeof(r));
    for (int k = 0; k < 2; k++) { r.status[k] = NotFound; r.location[k] = 0xffffffffu; r.direction[k] = 0; r.score[k] = -1; r.mapq[k] = 0; }
}
static void pairedPrint(const PairedAlignmentResult &r) {
    printf("\t%d\t%d\t%u\t%u\t%d\t%d\t%d\t%d\t%d\t%d", (int)r.status[0], (int)r.status[1], r.location[0], r.location[1],
           (int)r.direction[0], (int)r.direction[1], r.score[0], r.score[1], r.mapq[0], r.mapq[1]);
}
static int mode_paired(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "paired <indexDir> <reads0.fq> <reads1.fq> [maxHits maxK numSeeds extra minSpacing maxSpacing maxBigHits]\n"); return 2; }
    unsigned maxHits = argc > 5 ? atoi(argv[5]) : 16000;
    unsigned maxK = argc > 6 ? atoi(argv[6]) : 15;
    unsigned numSeeds = argc > 7 ? atoi(argv[7]) : 8;
    unsigned extra = argc > 8 ? atoi(argv[8]) : 2;
    unsigned minSpacing = argc > 9 ? atoi(argv[9]) : 50;
    unsigned maxSpacing = argc > 10 ? atoi(argv[10]) : 1000;
    unsigned maxBigHits = argc > 11 ? atoi(argv[11]) : DEFAULT_INTERSECTING_ALIGNER_MAX_HITS;
    const unsigned pool = DEFAULT_MAX_CANDIDATE_POOL_SIZE;
    initializeLVProbabilitiesToPhredPlus33();
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) { fprintf(stderr, "cannot load index %s\n", argv[2]); return 1; }
    const int maxReadSize = MAX_READ_LENGTH;
    BigAllocator *al = new BigAllocator(IntersectingPairedEndAligner::getBigAllocatorReservation(
        idx, maxBigHits, maxReadSize, idx->getSeedLength(), numSeeds, 0, maxK, extra, pool));
    IntersectingPairedEndAligner *ia = new IntersectingPairedEndAligner(idx, maxReadSize, maxHits, maxK, numSeeds, 0,
                                                                       minSpacing, maxSpacing, maxBigHits, extra, pool, al);
    ChimericPairedEndAligner *ca = new ChimericPairedEndAligner(idx, maxReadSize, maxHits, maxK, numSeeds, 0, minSpacing,
                                                               maxSpacing, false, extra, ia);
    std::ifstream in0(argv[3]), in1(argv[4]);
    std::string id[2], bases[2], plus[2], quals[2];
    unsigned i = 0;
    while (std::getline(in0, id[0]) && std::getline(in0, bases[0]) && std::getline(in0, plus[0]) && std::getline(in0, quals[0]) &&
           std::getline(in1, id[1]) && std::getline(in1, bases[1]) && std::getline(in1, plus[1]) && std::getline(in1, quals[1])) {
        std::string b[2], q[2];
        Read r[2];
        for (int k = 0; k < 2; k++) {
            b[k] = bases[k] + std::string(16, '\0');
            q[k] = quals[k] + std::string(16, '\0');
            r[k].init(id[k].c_str() + 1, (unsigned)id[k].size() - 1, b[k].c_str(), q[k].c_str(), (unsigned)bases[k].size());
        }
        PairedAlignmentResult res;
        printf("%u", i);
        pairedPre(res);
        _int64 s0 = ia->getLocationsScored();
        ia->align(&r[0], &r[1], &res);
        pairedPrint(res);
        printf("\t%lld", (long long)(ia->getLocationsScored() - s0));
        pairedPre(res);
        s0 = ca->getLocationsScored();
        ca->align(&r[0], &r[1], &res);
        pairedPrint(res);
        printf("\t%d\t%d\t%lld\n", (int)res.fromAlignTogether, (int)res.alignedAsPair, (long long)(ca->getLocationsScored() - s0));
        i++;
    }
    return 0;
}

static int mode_cigar(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "cigar <indexDir> <calls.tsv>\n"); return 2; }
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) return 1;
    const Genome *g = idx->getGenome();
    LandauVishkinWithCigar lvc;
    std::ifstream in(argv[3]);
    unsigned loc; int useM; int dirv; std::string read;
    char cig[MAX_READ_LENGTH * 2];
    while (in >> loc >> dirv >> useM >> read) {
        // getSAMData (SAM.cpp:866-883): Read::init upper-cases, RC = reversed COMPLEMENT[]
        Read r;
        r.init("x", 1, read.c_str(), read.c_str(), (unsigned)read.size());
        std::string p(read.size() + 16, '\0');
        for (size_t i = 0; i < read.size(); i++) {
            if (dirv) p[read.size() - 1 - i] = COMPLEMENT[(unsigned char)r.getData()[i]];
            else p[i] = r.getData()[i];
        }
        std::vector<unsigned> tokens;
        const char *ref = g->getSubstring(loc, (unsigned)read.size());
        if (ref == NULL) { printf("-3\t*\n"); continue; }
        int ed = lvc.computeEditDistance(ref, (int)read.size(), p.c_str(), (int)read.size(), MAX_K - 1,
                                         cig, sizeof(cig), useM != 0, tokens);
        printf("%d\t%s\n", ed, ed >= 0 ? cig : "*");
    }
    return 0;
}

static int mode_samheader(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "samheader <indexDir> <sorted> <version> [args...]\n"); return 2; }
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) return 1;
    ReaderContext ctx;
    memset(&ctx, 0, sizeof(ctx));
    ctx.genome = idx->getGenome();
    ctx.defaultReadGroup = "FASTQ";
    std::vector<char> buf(1 << 24);
    size_t used = 0;
    if (!FileFormat::SAM[0]->writeHeader(ctx, &buf[0], buf.size(), &used, atoi(argv[3]) != 0, argc - 5,
                                         (const char **)(argv + 5), argv[4], NULL)) return 1;
    fwrite(&buf[0], 1, used, stdout);
    return 0;
}

static void dumpSeedMap(const char *tag, seed_map &m) {
    printf("\t%s", tag);
    bool first = true;
    for (seed_map::iterator it = m.begin(); it != m.end(); ++it) {
        printf("%s%u:%u:%u:%u", first ? ":" : ",", it->first, *it->second.begin(), *it->second.rbegin(),
               (unsigned)it->second.size());
        first = false;
    }
}

static int mode_charseeds(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "charseeds <indexDir> <reads.fq> [maxHits maxK numSeeds extra]\n"); return 2; }
    unsigned maxHits = argc > 4 ? atoi(argv[4]) : 300;
    unsigned maxK = argc > 5 ? atoi(argv[5]) : 15;
    unsigned numSeeds = argc > 6 ? atoi(argv[6]) : 12;
    unsigned extra = argc > 7 ? atoi(argv[7]) : 2;
    initializeLVProbabilitiesToPhredPlus33();
    GenomeIndex *idx = GenomeIndex::loadFromDirectory(argv[2]);
    if (!idx) { fprintf(stderr, "cannot load index %s\n", argv[2]); return 1; }
    // the partial aligner of PairedAligner.cpp:518-527 (own LV objects, no BigAllocator)
    BaseAligner *ba = new BaseAligner(idx, maxHits, maxK, MAX_READ_LENGTH, numSeeds, 0, extra, NULL, NULL);
    std::ifstream in(argv[3]);
    std::string id, bases, plus, quals;
    unsigned i = 0;
    while (std::getline(in, id) && std::getline(in, bases) && std::getline(in, plus) && std::getline(in, quals)) {
        std::string b = bases + std::string(16, '\0');
        std::string q = quals + std::string(16, '\0');
        Read r;
        r.init(id.c_str() + 1, (unsigned)id.size() - 1, b.c_str(), q.c_str(), (unsigned)bases.size());
        seed_map map, mapRC;
        unsigned loc = InvalidGenomeLocation; Direction dir = 0; int score = 0, mapq = 0;
        ba->setReadId(0);
        ba->CharacterizeSeeds(&r, &loc, &dir, &score, &mapq, 0, 0, FORWARD, map, mapRC);
        printf("%u\t%u\t%u", i, (unsigned)map.size(), (unsigned)mapRC.size());
        dumpSeedMap("F", map);
        dumpSeedMap("RC", mapRC);
        printf("\n");
        i++;
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: ref_harness align|lv|lookup ...\n"); return 2; }
    std::string m = argv[1];
    if (m == "align") return mode_align(argc, argv);
    if (m == "alignx") return mode_alignx(argc, argv);
    if (m == "lv") return mode_lv(argc, argv);
    if (m == "lookup") return mode_lookup(argc, argv);
    if (m == "sam") return mode_sam(argc, argv);
    if (m == "cigar") return mode_cigar(argc, argv);
    if (m == "paired") return mode_paired(argc, argv);
    if (m == "samheader") return mode_samheader(argc, argv);
    if (m == "charseeds") return mode_charseeds(argc, argv);
    fprintf(stderr, "unknown mode %s\n", argv[1]);
    return 2;
}

/*
 * snap_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded-per-aligner restatement of the reference hot path
 *   BaseAligner::AlignRead        (SNAPLib/BaseAligner.cpp:510-938)
 *   BaseAligner::score            (SNAPLib/BaseAligner.cpp:977-1399)
 *   LandauVishkin<+-1>::computeEditDistance (SNAPLib/LandauVishkin.h:211-455)
 *   GenomeIndex::lookupSeed       (SNAPLib/GenomeIndex.cpp:971-1086)
 *   SNAPHashTable::Lookup         (SNAPLib/HashTable.h:74-105)
 *   computeMAPQ                   (SNAPLib/mapq.h:32-65)
 * used ONLY as the parity checker by tests/, __graft_entry__.smoke() and as the
 * `cpu_baseline` leg of bench.py.  The product path (snap-rnaseq_amd/) never
 * links or calls it.  Parity of this restatement is pinned against the
 * reference itself (oracle/_ref, built from /root/reference by
 * oracle/Makefile.ref) and the golden fixtures under tests/golden/.
 *
 * Data structures are deliberately different from both the reference (chained
 * anchors with epochs) and the GPU path (timestamped LDS arena): candidate
 * elements live in an open-addressed map keyed by (direction, 48-aligned
 * location) and the weight lists are explicit circular doubly-linked lists, the
 * FIFO order of the reference.
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "snapgpu.h"

#define MAX_K 31                 /* LandauVishkin.h:9 */
#define MAX_READ_LENGTH 500      /* Read.h:45 */
#define ELEM_SIZE 48             /* BaseAligner.h:163,196 maxMergeDist == hashTableElementSize */
#define UNUSED_SCORE 0xffffu     /* BaseAligner.h:261 */
#define INVALID_LOC 0xffffffffu  /* Genome.h:29 */
#define N_PADDING 100u           /* Genome.h:175 */
#define SNP_PROB 0.001           /* BaseAligner.h:264-266 */
#define GAP_OPEN_PROB 0.001
#define GAP_EXTEND_PROB 0.5
#define MAPQ_LIMIT_FOR_SINGLE_HIT 10   /* AlignerOptions.h:34 */

/* ---------------------------------------------------------------- tables */
/* initializeLVProbabilitiesToPhredPlus33 (LandauVishkin.cpp:601-649) */
static double g_indel[64];
static double g_phred[256];
static double g_perfect[MAX_READ_LENGTH + 1];
static double g_seedProb[33];    /* pow(1 - SNP_PROB, seedLen), BaseAligner.cpp:1227 */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* BaseAligner.cpp:1227 calls pow(double, int) with an `int seedLen`
 * (BaseAligner.cpp:1200).  The reference is C++98, where
 * libstdc++'s std::pow(double, int) is __builtin_powi, i.e. libgcc's __powidf2:
 * binary exponentiation by squaring -- NOT libm pow.  Restated here. */
static double powi_libgcc(double x, int m) {
    unsigned n = m < 0 ? -(unsigned)m : (unsigned)m;
    double y = (n % 2) ? x : 1;
    while (n >>= 1) {
        x = x * x;
        if (n % 2) y = y * x;
    }
    return m < 0 ? 1 / y : y;
}

static void init_tables(void) {
    g_indel[0] = 1.0;
    g_indel[1] = GAP_OPEN_PROB;
    for (int i = 2; i < 64; i++) g_indel[i] = g_indel[i - 1] * GAP_EXTEND_PROB;
    for (int i = 0; i < 33; i++) g_phred[i] = SNP_PROB;
    for (int i = 33; i <= 93 + 33; i++) g_phred[i] = 1.0 - (1.0 - pow(10.0, -1.0 * (i - 33.0) / 10.0)) * (1.0 - SNP_PROB);
    for (int i = 93 + 33 + 1; i < 256; i++) g_phred[i] = SNP_PROB;
    g_perfect[0] = 1.0;
    for (int i = 1; i <= MAX_READ_LENGTH; i++) g_perfect[i] = g_perfect[i - 1] * (1 - SNP_PROB);
    for (int i = 0; i < 33; i++) g_seedProb[i] = powi_libgcc(1 - SNP_PROB, i);
}

/* computeMAPQ, mapq.h:32-65 */
int oracle_compute_mapq(double pAll, double pBest, int score, int popular) {
    if (pAll < pBest) pAll = pBest;
    if (pAll == pBest && popular == 0 && score < 5) return 70;
    double c = pBest / pAll;
    int base;
    if (c >= 1) base = 69;
    else {
        base = (int)(-10 * log10(1 - c));
        if (base > 69) base = 69;
    }
    int pen = popular - 10;
    if (pen < 0) pen = 0;
    base -= pen / 2;
    return base < 0 ? 0 : base;
}

/* --------------------------------------------------------- Landau-Vishkin */
/* Text accessor: forward texts are read ascending from `text`; reverse texts are
 * read descending from text[-1] (LandauVishkin.h:261-263, 326, 336). */
static inline char lv_t(const char *text, int dir, int j) { return dir > 0 ? text[j] : text[-1 - j]; }


/* First m in [from, endd) with pattern[m] != T(m + d), else endd -- the
 * clipped result of the reference's 8-byte XOR/ctz loop (LandauVishkin.h:268-288,
 * 331-353). */
static inline int lv_extend(const char *text, int dir, const char *pattern, int m, int d, int endd) {
    while (m + 8 <= endd) {
        uint64_t pv, tv;
        memcpy(&pv, pattern + m, 8);
        if (dir > 0) memcpy(&tv, text + m + d, 8);
        else { memcpy(&tv, text - (m + d) - 8, 8); tv = __builtin_bswap64(tv); }
        uint64_t x = pv ^ tv;
        if (x) return m + (__builtin_ctzll(x) >> 3);
        m += 8;
    }
    while (m < endd && pattern[m] == lv_t(text, dir, m + d)) m++;
    return m;
}

/* LandauVishkin<dir>::computeEditDistance, LandauVishkin.h:211-455.  The 8-byte
 * XOR/ctz match extension is restated byte-wise: the reference clips every
 * extension with min(., end), so the bytes it over-reads past `end` only matter
 * through the `*p == *t` pre-test when best > end (kept below). */
int oracle_lv(int dir, const char *text, int textLen, const char *pattern, const char *qual,
              int patternLen, int k, double *prob, int *netIndel) {
    pthread_once(&g_once, init_tables);
    int L[MAX_K + 1][2 * MAX_K + 3];
    char A[MAX_K + 1][2 * MAX_K + 3];
    /* The reference fills L with -2 once (LandauVishkin.h:168) and row e only
     * ever writes |d| <= e, so every read outside the band sees -2.  Setting
     * just the cells row e reads outside row e-1's band is equivalent. */
    *netIndel = 0;
    if (k > MAX_K - 1) k = MAX_K - 1;
    if (!text) { *prob = 0.0; return -1; }
    *prob = 1.0;
    int end = patternLen < textLen ? patternLen : textLen;
    int i = lv_extend(text, dir, pattern, 0, 0, end);
    L[0][MAX_K] = i;
    if (i == end) {
        int result = patternLen > end ? patternLen - end : 0;
        *prob = g_perfect[patternLen];
        return result > k ? -1 : result;
    }
    for (int e = 1; e <= k; e++) {
        L[e - 1][MAX_K - e - 1] = L[e - 1][MAX_K - e] = -2;
        L[e - 1][MAX_K + e] = L[e - 1][MAX_K + e + 1] = -2;
        /* d order 0, 1, -1, 2, -2, ... (LandauVishkin.h:180-182, 311) */
        for (int j = 0; j < 2 * e + 1; j++) {
            int d = (j == 0) ? 0 : ((j & 1) ? (j + 1) / 2 : -(j / 2));
            int best = L[e - 1][MAX_K + d] + 1;
            char act = 'X';
            int left = L[e - 1][MAX_K + d - 1];
            if (left > best) { best = left; act = 'D'; }
            int right = L[e - 1][MAX_K + d + 1] + 1;
            if (right > best) { best = right; act = 'I'; }
            A[e][MAX_K + d] = act;
            int endd = patternLen < textLen - d ? patternLen : textLen - d;
            if (pattern[best] == lv_t(text, dir, best + d)) {
                if (best < endd) {
                    best = lv_extend(text, dir, pattern, best + 1, d, endd);
                } else {
                    best = endd;
                }
            }
            if (best == patternLen) {
                /* backtrace (LandauVishkin.h:376-431) */
                char bAct[MAX_K + 1];
                int bMatched[MAX_K + 1];
                L[e][MAX_K + d] = best;
                int curD = d;
                for (int ce = e; ce >= 1; ce--) {
                    char a = A[ce][MAX_K + curD];
                    bAct[ce] = a;
                    int src;
                    if (a == 'I') { src = curD + 1; bMatched[ce] = L[ce][MAX_K + curD] - L[ce - 1][MAX_K + src] - 1; }
                    else if (a == 'D') { src = curD - 1; bMatched[ce] = L[ce][MAX_K + curD] - L[ce - 1][MAX_K + src]; }
                    else { src = curD; bMatched[ce] = L[ce][MAX_K + curD] - L[ce - 1][MAX_K + src] - 1; }
                    curD = src;
                }
                double p = 1.0;
                int ce = 1, offset = L[0][MAX_K];
                while (ce <= e) {
                    char a = bAct[ce];
                    int cnt = 1;
                    while (ce + 1 <= e && bMatched[ce] == 0 && bAct[ce + 1] == a) { cnt++; ce++; }
                    if (a == 'I') { p *= g_indel[cnt]; offset += cnt; *netIndel += cnt; }
                    else if (a == 'D') { p *= g_indel[cnt]; offset -= cnt; *netIndel -= cnt; }
                    else {
                        for (int r = 0; r < cnt; r++) {
                            int qi = offset < 0 ? 0 : offset;
                            if (qi > patternLen - 1) qi = patternLen - 1;
                            p *= g_phred[(unsigned char)qual[qi]];
                            offset++;
                        }
                    }
                    offset += bMatched[ce];
                    ce++;
                }
                p *= g_perfect[patternLen - e];
                *prob = p;
                return e;
            }
            L[e][MAX_K + d] = best;
        }
    }
    return -1;
}

/* ------------------------------------------------------------ index view */
static inline uint32_t fmix32(uint32_t k) {   /* HashTable.h:60-72 */
    k ^= k >> 16; k *= 0x85ebca6bu; k ^= k >> 13; k *= 0xc2b2ae35u; k ^= k >> 16;
    return k;
}

/* SNAPHashTable::Lookup, HashTable.h:74-105 -> pointer to value1 or NULL */
static const uint32_t *ht_lookup(const snapgpu_index_view_t *v, uint32_t table, uint32_t key, uint32_t *probes) {
    uint64_t size = v->tableSize[table];
    const uint32_t *t = v->slots + 3 * v->tableBase[table];
    uint64_t i = fmix32(key) % size;
    *probes += 1;
    if (t[3 * i] == key && t[3 * i + 1] != INVALID_LOC) return t + 3 * i + 1;
    uint64_t n = 0;
    for (;;) {
        n++;
        if (n > size + 5) return NULL;
        i = (n < 5) ? (i + n * n) % size : (i + 1) % size;
        *probes += 1;
        if (t[3 * i] == key || t[3 * i + 1] == INVALID_LOC) break;
    }
    return t[3 * i + 1] == INVALID_LOC ? NULL : t + 3 * i + 1;
}

/* ------------------------------------------------------------- aligner */
typedef struct Elem {
    struct Elem *wnext, *wprev;
    uint64_t used, scored;
    uint32_t base, weight, lps, bestScore, bestLoc;
    int dir, allScored;
    double prob;
    int seedOffset[ELEM_SIZE];
} Elem;

typedef struct {
    uint32_t key;     /* (base/48) << 1 | dir, +1 so that 0 is empty */
    uint32_t epoch;
    Elem *elem;
} Slot;

typedef struct {
    const snapgpu_index_view_t *ix;
    snapgpu_aligner_params_t p;
    unsigned maxSeedsFromCmd, numWeightLists;
    Elem *pool; unsigned poolSize, nUsed;
    Slot *map; unsigned mapMask; uint32_t epoch;
    Elem *lists;                      /* sentinels [numWeightLists] */
    /* read buffers (+32 bytes of zero slack: LV over-reads, LandauVishkin.h:271) */
    char fwd[MAX_READ_LENGTH + 32], fwdQ[MAX_READ_LENGTH + 32];
    char rc[MAX_READ_LENGTH + 32], rcQ[MAX_READ_LENGTH + 32];
    char rev[2][MAX_READ_LENGTH + 32];
    uint8_t seedUsed[(MAX_READ_LENGTH + 7) / 8 + 8];
    /* per-read state, BaseAligner.h:273-289 */
    unsigned lps[2], mostSeeds[2], nSeedsApplied[2];
    unsigned bestScore, bestLoc, scoreLimit, popular;
    double pAll, pBest;
    snapgpu_result_t *out;
    /* multi-hit recording (BaseAligner.h:149-152) */
    unsigned maxHitsToGet;
    unsigned hitCount[MAX_K];
    unsigned hitSlot;                 /* distance stride: min(maxHitsToGet, 512) (BaseAligner.h:148-151) */
    uint32_t *hitLoc;                 /* [MAX_K * hitSlot + extra]: rows alias above 512 as the reference's */
    uint8_t *hitRC;
} Oracle;

static inline int base_value(char c) {   /* Tables.cpp:41-48 */
    switch (c) { case 'A': return 0; case 'G': return 1; case 'C': return 2; case 'T': return 3; default: return 4; }
}

static Elem *find_elem(Oracle *o, uint32_t loc, int dir) {   /* findElement, BaseAligner.cpp:1415-1442 */
    uint32_t base = loc - loc % ELEM_SIZE;
    uint32_t key = ((base / ELEM_SIZE) << 1 | (uint32_t)dir) + 1;
    uint32_t h = (key * 2654435761u) & o->mapMask;
    for (;;) {
        Slot *s = &o->map[h];
        if (s->epoch != o->epoch) return NULL;
        if (s->key == key) return s->elem;
        h = (h + 1) & o->mapMask;
    }
}

static void map_insert(Oracle *o, Elem *e) {
    uint32_t key = ((e->base / ELEM_SIZE) << 1 | (uint32_t)e->dir) + 1;
    uint32_t h = (key * 2654435761u) & o->mapMask;
    while (o->map[h].epoch == o->epoch) h = (h + 1) & o->mapMask;
    o->map[h].epoch = o->epoch; o->map[h].key = key; o->map[h].elem = e;
}

static inline void list_unlink(Elem *e) { e->wnext->wprev = e->wprev; e->wprev->wnext = e->wnext; }
static inline void list_append(Elem *sentinel, Elem *e) {
    e->wnext = sentinel; e->wprev = sentinel->wprev; e->wnext->wprev = e; e->wprev->wnext = e;
}

/* incrementWeight, BaseAligner.cpp:1689-1727 */
static void increment_weight(Oracle *o, Elem *e) {
    if (e->allScored) return;
    if (e->weight >= o->numWeightLists - 1) return;
    list_unlink(e);
    e->weight++;
    list_append(&o->lists[e->weight], e);
}

/* Genome::getSubstring, Genome.h:78-148 */
static const char *get_substring(const snapgpu_index_view_t *v, uint32_t offset, uint32_t len) {
    if (offset > v->nBases || (uint64_t)offset + len > (uint64_t)v->nBases + N_PADDING) return NULL;
    if (len <= v->chromosomePadding) return v->genome + offset;
    if (v->nPieces > 100) {
        if (v->pieceOffsets[v->nPieces - 1] <= offset) return v->genome + offset;
        int lo = 0, hi = v->nPieces - 2;
        while (lo <= hi) {
            int m = (lo + hi) / 2;
            if (v->pieceOffsets[m] <= offset) {
                if (v->pieceOffsets[m + 1] > offset)
                    return v->pieceOffsets[m + 1] <= offset + len - 1 ? NULL : v->genome + offset;
                lo = m + 1;
            } else hi = m - 1;
        }
        return NULL;
    }
    for (int i = 0; i < v->nPieces; i++)
        if (offset + len - 1 >= v->pieceOffsets[i]) return offset < v->pieceOffsets[i] ? NULL : v->genome + offset;
    return NULL;
}

static int next_piece_after(const snapgpu_index_view_t *v, uint32_t loc) {  /* Genome.cpp:376-401 */
    int lo = 0, hi = v->nPieces - 1;
    while (lo <= hi) {
        int m = (lo + hi) / 2;
        if (v->pieceOffsets[m] <= loc && (m == v->nPieces - 1 || v->pieceOffsets[m + 1] > loc))
            return m >= v->nPieces - 1 ? -1 : m + 1;
        else if (v->pieceOffsets[m] <= loc) lo = m + 1;
        else hi = m - 1;
    }
    return -1;
}

/* BaseAligner::score, BaseAligner.cpp:977-1399.  Returns 1 iff a result was reached. */
static int score(Oracle *o, int force, unsigned readLen, int *result) {
    snapgpu_result_t *out = o->out;
    const unsigned seedLen = o->ix->seedLen;
    for (int d = 0; d < 2; d++)
        if (o->mostSeeds[d]) {
            unsigned v = o->nSeedsApplied[d] / o->mostSeeds[d];
            if (v > o->lps[d]) o->lps[d] = v;
        }
    unsigned w = o->numWeightLists - 1;
    do {
        while (w > 0 && o->lists[w].wnext == &o->lists[w]) w--;
        unsigned minLps = o->lps[0] < o->lps[1] ? o->lps[0] : o->lps[1];
        if (minLps > o->scoreLimit || force) {
            if (w == 0) {
                out->score = (int)o->bestScore;
                if (o->bestScore <= o->p.maxK) {
                    out->location = o->bestLoc;
                    out->mapq = oracle_compute_mapq(o->pAll, o->pBest, (int)o->bestScore, (int)o->popular);
                    *result = out->mapq >= MAPQ_LIMIT_FOR_SINGLE_HIT ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
                } else {
                    *result = (o->nSeedsApplied[0] == 0 && o->nSeedsApplied[1] == 0) ? SNAPGPU_MULTIPLE_HITS : SNAPGPU_NOT_FOUND;
                    out->mapq = 0;
                }
                return 1;
            }
            force = 1;
        } else if (w == 0) {
            return 0;
        }
        Elem *el = o->lists[w].wnext;
        /* BaseAligner.cpp:1121-1127: prefetch the next element and its genome data */
        __builtin_prefetch(el->wnext->wnext);
        __builtin_prefetch(o->ix->genome + el->wnext->base);
        __builtin_prefetch(o->ix->genome + el->wnext->base + 64);
        if (el->lps <= o->scoreLimit) {
            uint64_t mask = el->used;
            while (mask) {
                unsigned bit = (unsigned)__builtin_ctzll(mask);
                uint64_t cbit = 1ull << bit;
                mask &= ~cbit;
                if (el->scored & cbit) continue;
                int anyNearby = el->scored != 0;
                el->scored |= cbit;
                uint32_t loc = el->base + bit;
                uint32_t elemLoc = loc;
                unsigned sc = 0xffffffffu;
                double prob = 0;
                const char *data = get_substring(o->ix, loc, readLen + MAX_K);
                unsigned gLen = readLen + MAX_K;
                if (!data) {   /* BaseAligner.cpp:1163-1185 */
                    uint32_t endOffset;
                    int np = -1;
                    if ((uint64_t)loc + readLen + MAX_K >= o->ix->nBases) endOffset = o->ix->nBases;
                    else { np = next_piece_after(o->ix, loc); endOffset = np >= 0 ? o->ix->pieceOffsets[np] : 0; }
                    if (np >= 0 || endOffset == o->ix->nBases) {
                        gLen = endOffset - loc - 1;
                        if (gLen >= readLen - (unsigned)MAX_K) data = get_substring(o->ix, loc, gLen);
                    }
                }
                if (data) {
                    const char *rd = el->dir ? o->rc : o->fwd;
                    const char *rq = el->dir ? o->rcQ : o->fwdQ;
                    const char *oppQ = el->dir ? o->fwdQ : o->rcQ;
                    int s = el->seedOffset[bit];
                    int tail = s + (int)seedLen;
                    double p1, p2; int ni1, ni2;
                    int s1 = oracle_lv(1, data + tail, (int)gLen - tail, rd + tail, rq + tail, (int)readLen - tail,
                                       (int)o->scoreLimit, &p1, &ni1);
                    if (s1 != -1) {
                        int limitLeft = (int)o->scoreLimit - s1;
                        int s2 = oracle_lv(-1, data + s, s + MAX_K, o->rev[el->dir] + readLen - s, oppQ + readLen - s, s,
                                           limitLeft, &p2, &ni2);
                        if (s2 != -1) {
                            sc = (unsigned)(s1 + s2);
                            prob = p1 * p2 * g_seedProb[seedLen];
                            loc += (uint32_t)ni2;
                        }
                    }
                }
                /* BaseAligner.cpp:1255-1261 */
                if (o->maxHitsToGet > 0 && sc != 0xffffffffu && sc < MAX_K && o->hitCount[sc] < o->maxHitsToGet) {
                    o->hitLoc[sc * o->hitSlot + o->hitCount[sc]] = loc;
                    o->hitRC[sc * o->hitSlot + o->hitCount[sc]] = (uint8_t)el->dir;
                    o->hitCount[sc]++;
                }
                out->nLocationsScored++;
                if (anyNearby) {
                    if (el->bestScore < sc || (el->bestScore == sc && prob <= el->prob)) continue;
                }
                el->bestLoc = loc;
                Elem *nb = NULL;
                if (sc != 0xffffffffu) {
                    uint32_t nl = elemLoc + (2 * (elemLoc % ELEM_SIZE / (ELEM_SIZE / 2)) - 1) * (ELEM_SIZE / 2);
                    nb = find_elem(o, nl, el->dir);
                }
                if (nb && nb->scored != 0) {
                    if (!((nb->base > el->base && loc - nb->bestLoc <= ELEM_SIZE) ||
                          (nb->base < el->base && nb->bestLoc <= ELEM_SIZE)))   /* sic, BaseAligner.cpp:1311-1312 */
                        nb = NULL;
                    if (nb) {
                        if (nb->bestScore < sc || (nb->bestScore == sc && nb->prob >= prob)) continue;
                        anyNearby = 1;
                        o->pAll = o->pAll - nb->prob > 0.0 ? o->pAll - nb->prob : 0.0;
                        nb->prob = 0;
                    }
                }
                o->pAll = o->pAll - el->prob > 0.0 ? o->pAll - el->prob : 0.0;
                o->pAll += prob;
                el->prob = prob;
                el->bestScore = sc;
                if (o->bestScore > sc || (o->bestScore == sc && prob > o->pBest)) {
                    o->bestScore = sc;
                    o->pBest = prob;
                    o->bestLoc = loc;
                    out->location = loc;
                    out->score = (int)sc;
                    out->direction = (uint8_t)el->dir;
                }
                if (o->p.stopOnFirstHit && o->bestScore <= o->p.maxK) {
                    *result = SNAPGPU_MULTIPLE_HITS;
                    out->mapq = 0;
                    return 1;
                }
                o->scoreLimit = (o->bestScore < o->p.maxK ? o->bestScore : o->p.maxK) + o->p.extraSearchDepth;
            }
        }
        el->allScored = 1;
        list_unlink(el);
        el->wnext = el->wprev = el;
    } while (force);
    return 0;
}

/* SeedSequencer.h:28-287, GetWrappedNextSeedToTest: the wrap order per seed length. */
static const unsigned char kWrap[10][25] = {
    /* 16 */ {0, 8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15},
    /* 17 */ {0, 8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15, 16},
    /* 18 */ {0, 9, 4, 13, 2, 6, 11, 15, 1, 3, 5, 7, 8, 10, 12, 14, 16, 17},
    /* 19 */ {0, 10, 4, 14, 2, 6, 8, 12, 16, 18, 1, 3, 5, 7, 9, 11, 13, 15, 17},
    /* 20 */ {0, 10, 5, 15, 2, 7, 12, 17, 3, 9, 11, 13, 19, 1, 4, 6, 8, 14, 18, 16},
    /* 21 */ {0, 11, 6, 16, 3, 9, 13, 17, 18, 2, 5, 8, 15, 20, 1, 4, 7, 10, 12, 14, 19},
    /* 22 */ {0, 11, 6, 16, 3, 9, 14, 19, 2, 7, 12, 17, 20, 4, 1, 10, 13, 15, 18, 21, 5, 8},
    /* 23 */ {0, 12, 6, 17, 3, 9, 20, 14, 1, 4, 7, 10, 15, 18, 21, 4, 2, 5, 11, 16, 19, 22, 8},
    /* 24 */ {0, 12, 6, 18, 3, 15, 21, 9, 1, 13, 19, 7, 16, 4, 22, 10, 2, 14, 20, 5, 17, 8, 23, 11},
    /* 25 */ {0, 13, 6, 19, 3, 16, 22, 9, 11, 1, 14, 7, 20, 4, 17, 23, 2, 15, 5, 21, 8, 24, 10, 18, 12},
};
static unsigned wrapped_next_seed(unsigned seedLen, unsigned wrapCount) {
    return kWrap[seedLen - 16][wrapCount];
}

/* BaseAligner::fillHitsFound, BaseAligner.cpp:940-975 */
static void fill_hits(Oracle *o, int32_t *found, snapgpu_multi_hit_t *mh) {
    if (o->maxHitsToGet == 0) return;
    *found = 0;
    unsigned first = 0;
    while (first < MAX_K && o->hitCount[first] == 0) first++;
    for (unsigned dist = first; dist < first + 4 && dist < MAX_K; dist++)
        for (unsigned i = 0; i < o->hitCount[dist]; i++) {
            mh[*found].location = o->hitLoc[dist * o->hitSlot + i];
            mh[*found].direction = o->hitRC[dist * o->hitSlot + i];
            mh[*found].score = (uint8_t)dist;
            mh[*found].reserved = 0;
            *found += 1;
            if ((unsigned)*found == o->maxHitsToGet) return;
        }
}

/* GenomeIndex::fillInLookedUpResults, GenomeIndex.cpp:1013-1086: the hits of one
 * side in [minLoc, maxLoc] (overflow lists are sorted descending). */
static void fill_side(const snapgpu_index_view_t *ix, uint32_t v, uint32_t minLoc, uint32_t maxLoc, uint32_t *single,
                      unsigned *nHits, const uint32_t **hits, uint32_t *nOvf) {
    if (v < ix->nBases) {
        *single = v;
        *nHits = (v >= minLoc && v <= maxLoc) ? 1 : 0;
        *hits = single;
    } else if (v == 0xfffffffeu) {
        *nHits = 0;
    } else {
        const uint32_t off = v - ix->nBases;
        const uint32_t cnt = ix->overflow[off];
        const uint32_t *all = ix->overflow + off + 1;
        (*nOvf)++;
        if (minLoc == 0 && maxLoc == INVALID_LOC) { *nHits = cnt; *hits = all; return; }
        unsigned lo = 0, hi = cnt;   /* first index with all[i] <= maxLoc */
        while (lo < hi) { unsigned m = (lo + hi) / 2; if (all[m] <= maxLoc) hi = m; else lo = m + 1; }
        unsigned end = lo;
        while (end < cnt && all[end] >= minLoc) end++;
        *nHits = end - lo;
        *hits = all + lo;
    }
}

/* BaseAligner::AlignRead, BaseAligner.cpp:510-938 */
static void align_read(Oracle *o, const char *bases, const char *quals, unsigned readLen, snapgpu_result_t *out,
                       const snapgpu_search_t *search, int32_t *multiFound, snapgpu_multi_hit_t *multiHits) {
    const snapgpu_index_view_t *ix = o->ix;
    const unsigned seedLen = ix->seedLen;
    memset(out, 0, sizeof(*out));
    o->out = out;
    unsigned maxSeeds = o->maxSeedsFromCmd ? o->maxSeedsFromCmd
                                           : (unsigned)(int)(o->p.maxSeedCoverage * readLen / seedLen);
    out->location = INVALID_LOC;
    out->direction = SNAPGPU_FORWARD;
    out->score = (int)UNUSED_SCORE;
    o->popular = 0;
    o->pAll = o->pBest = 0;
    if (o->maxHitsToGet > 0) { memset(o->hitCount, 0, sizeof(o->hitCount)); *multiFound = 0; }
    /* search window, BaseAligner.cpp:596-602 */
    const uint32_t radius = search ? search->searchRadius : 0;
    uint32_t minLocation = 0, maxLocation = INVALID_LOC;
    if (radius != 0) {
        minLocation = search->searchLocation > radius ? search->searchLocation - radius : 0;
        maxLocation = search->searchLocation < INVALID_LOC - radius ? search->searchLocation + radius : INVALID_LOC;
    }
    if (readLen > o->p.maxReadSize) { out->flags |= SNAPGPU_FLAG_READ_TOO_LONG; out->result = SNAPGPU_NOT_FOUND; return; }
    if ((int)readLen < (int)seedLen) { out->result = SNAPGPU_NOT_FOUND; return; }
    /* Read::init upper-cases (Read.h:303-325); RC / reversed copies (BaseAligner.cpp:636-650) */
    unsigned countOfNs = 0;
    for (unsigned i = 0; i < readLen; i++) {
        char c = bases[i];
        if (c >= 'a' && c <= 'z') c = (char)(c - 0x20);
        char comp = c == 'A' ? 'T' : c == 'G' ? 'C' : c == 'C' ? 'G' : c == 'T' ? 'A' : c == 'N' ? 'N' : 0;
        o->fwd[i] = c; o->fwdQ[i] = quals[i];
        o->rc[readLen - i - 1] = comp; o->rcQ[readLen - i - 1] = quals[i];
        o->rev[0][readLen - i - 1] = c;
        o->rev[1][i] = comp;
        countOfNs += c == 'N';
    }
    memset(o->fwd + readLen, 0, 32); memset(o->fwdQ + readLen, 0, 32);
    memset(o->rc + readLen, 0, 32); memset(o->rcQ + readLen, 0, 32);
    memset(o->rev[0] + readLen, 0, 32); memset(o->rev[1] + readLen, 0, 32);
    if (countOfNs > o->p.maxK) { out->flags |= SNAPGPU_FLAG_TOO_MANY_NS; out->result = SNAPGPU_NOT_FOUND; return; }
    /* clearCandidates, BaseAligner.cpp:1679-1687 */
    o->epoch++;
    o->nUsed = 0;
    for (unsigned i = 1; i < o->numWeightLists; i++) o->lists[i].wnext = o->lists[i].wprev = &o->lists[i];
    memset(o->seedUsed, 0, sizeof(o->seedUsed));
    unsigned nPossible = readLen - seedLen + 1, next = 0, wrapCount = 0;
    o->lps[0] = o->lps[1] = 0;
    o->mostSeeds[0] = o->mostSeeds[1] = 1;
    o->bestScore = UNUSED_SCORE;
    o->nSeedsApplied[0] = o->nSeedsApplied[1] = 0;
    o->scoreLimit = o->p.maxK + o->p.extraSearchDepth;
    int result = SNAPGPU_NOT_FOUND;
    while (o->nSeedsApplied[0] + o->nSeedsApplied[1] < maxSeeds) {
        if (next >= nPossible) {
            wrapCount++;
            if (wrapCount >= seedLen) {
                score(o, 1, readLen, &result);
                goto finish;
            }
            next = wrapped_next_seed(seedLen, wrapCount);
            o->mostSeeds[0] = o->mostSeeds[1] = wrapCount + 1;
        }
        while (next < nPossible && (o->seedUsed[next / 8] & (1 << (next % 8)))) next++;
        if (next >= nPossible) continue;
        o->seedUsed[next / 8] |= (uint8_t)(1 << (next % 8));
        /* Seed::DoesTextRepresentASeed + Seed::Seed (Seed.cpp:28-42, Seed.h:38-51) */
        uint64_t f = 0, r = 0;
        int valid = 1;
        for (unsigned i = 0; i < seedLen; i++) {
            int v = base_value(o->fwd[next + i]);
            if (v > 3) { valid = 0; break; }
            f |= (uint64_t)v << ((seedLen - i - 1) * 2);
            r |= (uint64_t)(v ^ 3) << (i * 2);
        }
        if (!valid) continue;
        /* GenomeIndex::lookupSeed, GenomeIndex.cpp:971-1011, windowed as BaseAligner.cpp:781-783 */
        const uint32_t minSeedLoc = minLocation < readLen ? 0 : minLocation - readLen;
        const uint32_t maxSeedLoc = maxLocation > INVALID_LOC - readLen ? INVALID_LOC : maxLocation + readLen;
        unsigned nHits[2] = {0, 0};
        const uint32_t *hits[2] = {NULL, NULL};
        uint32_t singleton[2];
        int comp = (int64_t)f > (int64_t)r;
        uint64_t canon = comp ? r : f;
        const uint32_t *e = ht_lookup(ix, (uint32_t)(canon >> 32), (uint32_t)canon, &out->nProbes);
        if (e) {
            for (int side = 0; side < 2; side++) {
                uint32_t v = (side == 0) == !comp ? e[0] : e[1];   /* fwd: value1 unless complemented */
                if (side == 1 && f == r) { nHits[1] = nHits[0]; hits[1] = hits[0]; break; }
                fill_side(ix, v, minSeedLoc, maxSeedLoc, &singleton[side], &nHits[side], &hits[side],
                          &out->nOverflowLists);
            }
        }
        out->nLookups++;
        int applied = 0;
        for (int dir = 0; dir < 2; dir++) {
            if (radius != 0 && (uint32_t)dir != search->searchDirection) continue;   /* BaseAligner.cpp:804-809 */
            if (nHits[dir] > o->p.maxHitsToConsider && !o->p.explorePopularSeeds) {
                out->nHitsIgnored++;
                o->popular++;
            } else {
                unsigned offset = dir == 0 ? next : readLen - seedLen - next;
                unsigned lim = nHits[dir] < o->p.maxHitsToConsider ? nHits[dir] : o->p.maxHitsToConsider;
                out->nHitWords += lim;
                for (unsigned i = 0; i < lim; i++) {
                    if (i % 16 == 0) {   /* prefetch candidate-map slots (BaseAligner.cpp:829-842) */
                        for (unsigned j = i; j < i + 16 && j < lim; j++) {
                            uint32_t l2 = hits[dir][j] - offset;
                            uint32_t key = (((l2 - l2 % ELEM_SIZE) / ELEM_SIZE) << 1 | (uint32_t)dir) + 1;
                            __builtin_prefetch(&o->map[(key * 2654435761u) & o->mapMask]);
                        }
                    }
                    uint32_t h = hits[dir][i];
                    uint32_t loc = h - offset;
                    if (loc < minLocation || loc > maxLocation || h < offset) continue;   /* BaseAligner.cpp:849-853 */
                    Elem *el = find_elem(o, loc, dir);
                    unsigned bit = loc % ELEM_SIZE;
                    if (el) {
                        /* findCandidate (BaseAligner.cpp:1474-1479) then incrementWeight */
                        uint64_t cb = 1ull << bit;
                        el->allScored = el->allScored && (el->used & cb);
                        el->used |= cb;
                        increment_weight(o, el);
                        el->seedOffset[bit] = (int)offset;
                    } else if (o->lps[dir] <= o->scoreLimit) {
                        /* allocateNewCandidate, BaseAligner.cpp:1485-1568 */
                        el = &o->pool[o->nUsed++];
                        out->nElements++;
                        el->used = 1ull << bit;
                        el->scored = 0;
                        el->lps = o->lps[dir];
                        el->dir = dir;
                        el->weight = 1;
                        el->base = loc - bit;
                        el->bestScore = UNUSED_SCORE;
                        el->allScored = 0;
                        el->prob = 0;
                        list_append(&o->lists[1], el);
                        el->seedOffset[bit] = (int)offset;
                        map_insert(o, el);
                    }
                }
                o->nSeedsApplied[dir]++;
                applied = 1;
            }
        }
        next += seedLen;
        if (applied && score(o, 0, readLen, &result)) { fill_hits(o, multiFound, multiHits); goto finish; }
    }
    score(o, 1, readLen, &result);
    fill_hits(o, multiFound, multiHits);   /* (not on the wrap-count exit above, BaseAligner.cpp:697-719) */
finish:
    out->result = (uint8_t)result;
    out->popularSeedsSkipped = (uint16_t)o->popular;
    out->probabilityOfAllCandidates = o->pAll;
    out->probabilityOfBestCandidate = o->pBest;
}

static Oracle *oracle_new(const snapgpu_index_view_t *ix, const snapgpu_aligner_params_t *p, unsigned maxHitsToGet) {
    pthread_once(&g_once, init_tables);
    Oracle *o = (Oracle *)calloc(1, sizeof(Oracle));
    o->ix = ix;
    o->p = *p;
    o->maxSeedsFromCmd = p->maxSeedsToUse;
    unsigned maxSeeds = p->maxSeedsToUse ? p->maxSeedsToUse
                                         : (unsigned)(int)(p->maxSeedCoverage * p->maxReadSize / ix->seedLen);
    o->numWeightLists = maxSeeds + 1;   /* BaseAligner.cpp:120-127 */
    o->poolSize = p->maxHitsToConsider * maxSeeds * 2 + 2 * p->maxHitsToConsider + 64;
    o->pool = (Elem *)calloc(o->poolSize, sizeof(Elem));
    unsigned m = 1;
    while (m < 2 * o->poolSize) m <<= 1;
    o->map = (Slot *)calloc(m, sizeof(Slot));
    o->mapMask = m - 1;
    o->lists = (Elem *)calloc(o->numWeightLists + 1, sizeof(Elem));
    for (unsigned i = 0; i <= o->numWeightLists; i++) o->lists[i].wnext = o->lists[i].wprev = &o->lists[i];
    o->maxHitsToGet = maxHitsToGet;
    if (maxHitsToGet) {
        o->hitSlot = maxHitsToGet < 512 ? maxHitsToGet : 512;
        const size_t cells = (size_t)MAX_K * o->hitSlot + (maxHitsToGet > 512 ? maxHitsToGet : 0);
        o->hitLoc = (uint32_t *)calloc(cells, sizeof(uint32_t));
        o->hitRC = (uint8_t *)calloc(cells, 1);
    }
    return o;
}

static void oracle_delete(Oracle *o) {
    free(o->pool); free(o->map); free(o->lists); free(o->hitLoc); free(o->hitRC); free(o);
}

typedef struct {
    const snapgpu_index_view_t *ix;
    const snapgpu_aligner_params_t *p;
    const char *bases, *quals;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint64_t n;
    snapgpu_result_t *out;
    volatile uint64_t *cursor;
    const snapgpu_search_t *search;
    unsigned maxHitsToGet;
    int32_t *multiFound;
    snapgpu_multi_hit_t *multiHits;
} Job;

static void *worker(void *arg) {
    Job *j = (Job *)arg;
    Oracle *o = oracle_new(j->ix, j->p, j->maxHitsToGet);
    for (;;) {
        uint64_t b = __atomic_fetch_add(j->cursor, 64, __ATOMIC_RELAXED);
        if (b >= j->n) break;
        uint64_t e = b + 64 < j->n ? b + 64 : j->n;
        for (uint64_t i = b; i < e; i++)
            align_read(o, j->bases + j->offsets[i], j->quals + j->offsets[i], j->lengths[i], &j->out[i],
                       j->search ? &j->search[i] : NULL, j->multiFound ? &j->multiFound[i] : NULL,
                       j->multiHits ? j->multiHits + i * j->maxHitsToGet : NULL);
    }
    oracle_delete(o);
    return NULL;
}

/* Align a batch of reads on `nThreads` host threads (one private aligner each,
 * as ParallelTask gives each thread its own BaseAligner, ParallelTask.h:127-137). */
int oracle_align_batch_ex(const snapgpu_index_view_t *ix, const snapgpu_aligner_params_t *p,
                          const char *bases, const char *quals, const uint64_t *offsets, const uint32_t *lengths,
                          uint64_t n, const snapgpu_search_t *search, unsigned maxHitsToGet, snapgpu_result_t *out,
                          int32_t *multiFound, snapgpu_multi_hit_t *multiHits, int nThreads) {
    if (ix->seedLen < 16 || ix->seedLen > 25) return -1;
    if (maxHitsToGet && (!multiFound || !multiHits)) return -1;
    if (nThreads < 1) nThreads = 1;
    volatile uint64_t cursor = 0;
    Job job = {ix, p, bases, quals, offsets, lengths, n, out, &cursor, search, maxHitsToGet, multiFound, multiHits};
    pthread_t *th = (pthread_t *)calloc((size_t)nThreads, sizeof(pthread_t));
    for (int t = 0; t < nThreads; t++) pthread_create(&th[t], NULL, worker, &job);
    for (int t = 0; t < nThreads; t++) pthread_join(th[t], NULL);
    free(th);
    return 0;
}

int oracle_align_batch(const snapgpu_index_view_t *ix, const snapgpu_aligner_params_t *p,
                       const char *bases, const char *quals, const uint64_t *offsets, const uint32_t *lengths,
                       uint64_t n, snapgpu_result_t *out, int nThreads) {
    return oracle_align_batch_ex(ix, p, bases, quals, offsets, lengths, n, NULL, 0, out, NULL, NULL, nThreads);
}

/* ------------------------------------------------------------------ CIGAR */
/* LandauVishkinWithCigar::computeEditDistance (LandauVishkin.cpp:252-535) as
 * SAMFormat::computeCigarString (SAM.cpp:1162-1230) calls it: text = the genome
 * substring at `loc` of the read's length, k = MAX_K - 1, COMPACT format.  Ops are
 * written as BAM ops (count << 4 | code, code index into "MIDNSHP=X"); `pattern`
 * must carry >= 8 bytes of zero slack (the reference compares 8 bytes at a time).
 * Returns the edit distance (NM), or -1 for "*" (no substring, or no alignment
 * within k).  A serial restatement: explicit L/A tables, diagonals visited in the
 * reference's order 0, -1, +1, -2, +2, ... */
static void cig_put(uint32_t *ops, int *n, int count, char c) {   /* writeCigar, LandauVishkin.cpp:27-93 */
    if (count <= 0) return;
    int code = c == 'M' ? 0 : c == 'I' ? 1 : c == 'D' ? 2 : c == '=' ? 7 : 8;
    ops[(*n)++] = ((uint32_t)count << 4) | (uint32_t)code;
}

int oracle_cigar(const snapgpu_index_view_t *v, uint32_t loc, const char *pattern, int len, int useM,
                 uint32_t *ops, int *nOps) {
    *nOps = 0;
    const char *text = get_substring(v, loc, (uint32_t)len);
    if (!text) return -1;
    const int k = MAX_K - 1;
    int L[MAX_K + 1][2 * MAX_K + 1];
    char A[MAX_K + 1][2 * MAX_K + 1];
    for (int i = 0; i <= MAX_K; i++)
        for (int j = 0; j <= 2 * MAX_K; j++) L[i][j] = -2;
    const int end = len;                       /* min(patternLen, textLen) */
    int m0 = 0;
    while (m0 < end && pattern[m0] == text[m0]) m0++;
    L[0][MAX_K] = m0;
    if (m0 == end) {
        cig_put(ops, nOps, len, useM ? 'M' : '=');
        return 0;
    }
    for (int e = 1; e <= k; e++) {
        for (int d = 0; d != -(e + 1); d = (d >= 0 ? -(d + 1) : -d)) {
            int best = L[e - 1][MAX_K + d] + 1;
            char a = 'X';
            int left = L[e - 1][MAX_K + d - 1];
            if (left > best) { best = left; a = 'D'; }
            int right = L[e - 1][MAX_K + d + 1] + 1;
            if (right > best) { best = right; a = 'I'; }
            A[e][MAX_K + d] = a;
            if (pattern[best] == text[d + best]) {
                int endd = len < len - d ? len : len - d;
                int m = best;
                while (m < endd && pattern[m] == text[d + m]) m++;
                best = m < endd ? m : endd;
            }
            L[e][MAX_K + d] = best;
            if (best != len) continue;
            /* done at (e, d): straight alignment with e mismatches? (LandauVishkin.cpp:341-393) */
            int straight = 0;
            for (int i = 0; i < end; i++) straight += pattern[i] != text[i];
            if (straight == e) {
                if (useM) { cig_put(ops, nOps, len, 'M'); return e; }
                int streak = 0, matching = pattern[0] == text[0];
                for (int i = 0; i < end; i++) {
                    int nm = pattern[i] == text[i];
                    if (nm != matching) { cig_put(ops, nOps, i - streak, matching ? '=' : 'X'); matching = nm; streak = i; }
                }
                if (len > streak) cig_put(ops, nOps, len - streak, matching ? '=' : 'X');
                return e;
            }
            /* backtrace (LandauVishkin.cpp:420-440) and emission (:442-520) */
            char act[MAX_K + 1]; int matched[MAX_K + 1];
            int curD = d;
            for (int ce = e; ce >= 1; ce--) {
                act[ce] = A[ce][MAX_K + curD];
                int pd = act[ce] == 'I' ? curD + 1 : act[ce] == 'D' ? curD - 1 : curD;
                matched[ce] = L[ce][MAX_K + curD] - L[ce - 1][MAX_K + pd] - (act[ce] == 'D' ? 0 : 1);
                curD = pd;
            }
            int accM = 0;
            if (useM) accM = L[0][MAX_K];
            else if (L[0][MAX_K] > 0) cig_put(ops, nOps, L[0][MAX_K], '=');
            for (int ce = 1; ce <= e; ce++) {
                char a2 = act[ce];
                int cnt = 1;
                while (ce + 1 <= e && matched[ce] == 0 && act[ce + 1] == a2) { cnt++; ce++; }
                if (useM) {
                    if (a2 == 'X') accM += cnt;
                    else { if (accM) { cig_put(ops, nOps, accM, 'M'); accM = 0; } cig_put(ops, nOps, cnt, a2); }
                } else cig_put(ops, nOps, cnt, a2);
                if (matched[ce] > 0) {
                    if (useM) accM += matched[ce];
                    else cig_put(ops, nOps, matched[ce], '=');
                }
            }
            if (useM && accM) cig_put(ops, nOps, accM, 'M');
            return e;
        }
    }
    return -1;
}

/* ============================================================== paired-end (f2)
 * IntersectingPairedEndAligner::align (IntersectingPairedEndAligner.cpp:142-753) and
 * ChimericPairedEndAligner::align (ChimericPairedEndAligner.cpp:56-126), restated over the
 * helpers above (lookup, LV, getSubstring, BaseAligner for the chimeric fallback).
 * The hit sets (HashTableHitSet, :844-1322, the "traditional" binary search of :1219-1263),
 * the mate / candidate pools and the merge anchors are plain arrays here.  Unsigned
 * arithmetic is kept where the reference's comparisons depend on it. */
#define P_MAX_SEEDS 30            /* IntersectingPairedEndAligner.h:93 MAX_MAX_SEEDS */
#define P_LOOKUP_CAP 64           /* lookups per hit set (seedCoverage mode can ask for more than 30) */

/* isWithin, Util.h:538-541 */
static inline int is_within(uint32_t a, uint32_t b, uint32_t d) { return (a <= b && a + d >= b) || (a >= b && a <= b + d); }
static inline uint32_t loc_distance(uint32_t a, uint32_t b) { return a > b ? a - b : b - a; }   /* Genome.cpp:473-479 */

typedef struct {
    uint32_t seedOffset, nHits, cur, set;
    const uint32_t *hits;
    uint32_t single;              /* the singleton a slot value holds (hits points here) */
} PLookup;

typedef struct {                  /* HashTableHitSet */
    PLookup lk[P_LOOKUP_CAP];
    unsigned nLookups, maxMerge;
    int curSet;
    unsigned exhausted[P_LOOKUP_CAP], miss[P_LOOKUP_CAP];
    uint32_t lastReturned;        /* mostRecentLocationReturned */
} PHitSet;

static void hs_record(PHitSet *h, uint32_t seedOffset, unsigned nHits, const uint32_t *hits, uint32_t single, int begins) {
    if (begins) { h->curSet++; h->exhausted[h->curSet] = 0; }                 /* :863-867 */
    if (nHits == 0) { h->exhausted[h->curSet]++; return; }
    PLookup *l = &h->lk[h->nLookups++];
    l->cur = 0; l->nHits = nHits; l->seedOffset = seedOffset; l->set = (uint32_t)h->curSet;
    l->single = single;
    l->hits = nHits == 1 && hits == NULL ? &l->single : hits;
    while (l->nHits > 0 && l->hits[l->nHits - 1] < l->seedOffset) l->nHits--;   /* :882-884 */
}

static unsigned hs_best_possible(PHitSet *h) {   /* computeBestPossibleScoreForCurrentHit, :901-929 */
    for (int i = 0; i <= h->curSet; i++) h->miss[i] = h->exhausted[i];
    for (unsigned i = 0; i < h->nLookups; i++) {
        PLookup *l = &h->lk[i];
        uint32_t target = h->lastReturned + l->seedOffset;
        int near = (l->cur != l->nHits && is_within(l->hits[l->cur], target, h->maxMerge)) ||
                   (l->cur != 0 && is_within(l->hits[l->cur - 1], target, h->maxMerge));
        if (!near) h->miss[l->set]++;
    }
    unsigned best = 0;
    for (int i = 0; i <= h->curSet; i++) if (h->miss[i] > best) best = h->miss[i];
    return best;
}

/* getNextHitLessThanOrEqualTo, the traditional version (:1219-1266) */
static int hs_next_le(PHitSet *h, uint32_t maxOff, uint32_t *loc, uint32_t *seedOff) {
    int any = 0;
    uint32_t bestOff = 0;
    for (unsigned i = 0; i < h->nLookups; i++) {
        PLookup *l = &h->lk[i];
        int lim0 = (int)l->cur, lim1 = (int)l->nHits - 1;
        uint32_t maxThis = maxOff + l->seedOffset;
        while (lim0 <= lim1) {
            unsigned probe = (unsigned)(lim0 + lim1) / 2;
            if (l->hits[probe] <= maxThis && (probe == 0 || l->hits[probe - 1] > maxThis)) {
                if (l->hits[probe] - l->seedOffset > bestOff) {
                    any = 1;
                    h->lastReturned = *loc = bestOff = l->hits[probe] - l->seedOffset;
                    *seedOff = l->seedOffset;
                }
                l->cur = probe;
                break;
            }
            if (l->hits[probe] > maxThis) lim0 = (int)probe + 1;
            else lim1 = (int)(probe - 1);
        }
        if (lim0 > lim1) l->cur = l->nHits;
    }
    return any;
}

static int hs_first(PHitSet *h, uint32_t *loc, uint32_t *seedOff) {   /* getFirstHit, :1270-1284 */
    int any = 0;
    *loc = 0;
    for (unsigned i = 0; i < h->nLookups; i++) {
        PLookup *l = &h->lk[i];
        if (l->nHits > 0 && l->hits[0] - l->seedOffset > *loc) {
            h->lastReturned = *loc = l->hits[0] - l->seedOffset;
            *seedOff = l->seedOffset;
            any = 1;
        }
    }
    return any;
}

static int hs_next_lower(PHitSet *h, uint32_t *loc, uint32_t *seedOff) {   /* getNextLowerHit, :1286-1322 */
    uint32_t found = 0;
    int any = 0;
    for (unsigned i = 0; i < h->nLookups; i++) {
        PLookup *l = &h->lk[i];
        if (l->cur != l->nHits && l->hits[l->cur] - l->seedOffset == h->lastReturned) l->cur++;
        if (l->cur != l->nHits && found < l->hits[l->cur] - l->seedOffset && l->hits[l->cur] >= l->seedOffset) {
            *loc = found = l->hits[l->cur] - l->seedOffset;
            *seedOff = l->seedOffset;
            any = 1;
        }
    }
    if (any) h->lastReturned = found;
    return any;
}

typedef struct {                  /* ScoringMateCandidate, IntersectingPairedEndAligner.h:401-423 */
    double prob;
    uint32_t loc, bestPossible, score, scoreLimit, seedOffset;
    int genomeOffset;
} PMate;
typedef struct {                  /* ScoringCandidate, :425-447 (indices instead of pointers) */
    int next, anchor;
    uint32_t mateIndex, loc, setPair, seedOffset, bestPossible;
} PCand;
typedef struct {                  /* MergeAnchor, :364-393 */
    double prob;
    uint32_t moreLoc, fewerLoc;
    int pairScore;
} PAnchor;

typedef struct {
    const snapgpu_index_view_t *ix;
    snapgpu_paired_params_t p;
    unsigned maxSeedsCmd, poolSize;
    PHitSet hs[2][2];
    PCand *cand; PMate *mate[2]; PAnchor *anchor;
    int *lists;                   /* scoringCandidates[maxK + extra + 1] */
    char data[2][2][MAX_READ_LENGTH + 32], qual[2][2][MAX_READ_LENGTH + 32], rev[2][2][MAX_READ_LENGTH + 32];
    unsigned len[2];
    uint32_t nScored;
    Oracle *single;               /* the chimeric fallback's BaseAligner */
} POracle;

/* scoreLocation, IntersectingPairedEndAligner.cpp:755-841 */
static void p_score_location(POracle *o, unsigned r, int dir, uint32_t loc, uint32_t seedOffset, uint32_t scoreLimit,
                             uint32_t *score, double *prob, int *offset) {
    const snapgpu_index_view_t *ix = o->ix;
    o->nScored++;
    const unsigned n = o->len[r];
    uint32_t gLen = n + MAX_K;
    const char *data = get_substring(ix, loc, gLen);
    if (!data) {
        uint32_t endOffset;
        if ((uint64_t)loc + n + MAX_K >= ix->nBases) endOffset = ix->nBases;
        else {   /* getPieceAtLocation(loc + n + MAX_K)->beginningOffset (Genome.cpp:356-374) */
            uint32_t at = loc + n + MAX_K;
            int lo = 0, hi = ix->nPieces - 1, pc = -1;
            while (lo <= hi) {
                int m = (lo + hi) / 2;
                if (ix->pieceOffsets[m] <= at && (m == ix->nPieces - 1 || ix->pieceOffsets[m + 1] > at)) { pc = m; break; }
                else if (ix->pieceOffsets[m] <= at) lo = m + 1;
                else hi = m - 1;
            }
            endOffset = pc >= 0 ? ix->pieceOffsets[pc] : 0;
        }
        gLen = endOffset - loc - 1;
        if (gLen >= n - (uint32_t)MAX_K) data = get_substring(ix, loc, gLen);
    }
    if (!data) { *score = 0xffffffffu; *prob = 0; return; }
    const int seedLen = (int)ix->seedLen, tail = (int)seedOffset + seedLen;
    double p1 = 0, p2 = 0;
    int ni;
    int s1 = oracle_lv(1, data + tail, (int)gLen - tail, o->data[r][dir] + tail, o->qual[r][dir] + tail, (int)n - tail,
                       (int)scoreLimit, &p1, &ni);
    if (s1 == -1) *score = 0xffffffffu;
    else {
        int limitLeft = (int)scoreLimit - s1;
        int s2 = oracle_lv(-1, data + seedOffset, (int)seedOffset + MAX_K, o->rev[r][dir] + n - seedOffset,
                           o->qual[r][!dir] + n - seedOffset, (int)seedOffset, limitLeft, &p2, offset);
        if (s2 == -1) *score = 0xffffffffu;
        else {
            *score = (uint32_t)(s1 + s2);
            *prob = p1 * p2 * g_seedProb[seedLen];
        }
    }
    if (*score == 0xffffffffu) *prob = 0;
}

static void pair_pre(snapgpu_pair_result_t *r) {
    memset(r, 0, sizeof(*r));
    for (int k = 0; k < 2; k++) { r->location[k] = INVALID_LOC; r->score[k] = -1; }
}

/* IntersectingPairedEndAligner::align; returns 0, or -1 when the reference would soft_exit */
static int p_align(POracle *o, const char *b0, const char *q0, unsigned n0, const char *b1, const char *q1, unsigned n1,
                   snapgpu_pair_result_t *res) {
    const snapgpu_index_view_t *ix = o->ix;
    const unsigned seedLen = ix->seedLen;
    const unsigned maxK = o->p.maxK, extra = o->p.extraSearchDepth;
    const char *B[2] = {b0, b1}, *Q[2] = {q0, q1};
    unsigned N[2] = {n0, n1};
    o->nScored = 0;
    unsigned maxSeeds = o->maxSeedsCmd ? o->maxSeedsCmd
                                       : (unsigned)((n0 > n1 ? n0 : n1) * o->p.seedCoverage / seedLen);   /* :150-155 */
    for (unsigned k = 0; k <= maxK + extra; k++) o->lists[k] = -1;
    unsigned nCand = 0, nMate[2] = {0, 0}, nAnchor = 0;
    if (n0 < 50 || n1 < 50) return 0;                                         /* :186-188 */
    unsigned countOfNs = 0, popular[2] = {0, 0}, nLookups[2] = {0, 0}, total[2][2] = {{0, 0}, {0, 0}};
    for (unsigned r = 0; r < 2; r++) {
        o->len[r] = N[r];
        for (int d = 0; d < 2; d++) {
            PHitSet *h = &o->hs[r][d];
            h->nLookups = 0; h->curSet = -1; h->maxMerge = maxK;               /* firstInit(maxSeeds, maxK), init() */
        }
        if (N[r] > o->p.maxReadSize) { res->flags |= SNAPGPU_PFLAG_READ_TOO_LONG; return -1; }
        for (unsigned i = 0; i < N[r]; i++) {
            char c = B[r][i];
            if (c >= 'a' && c <= 'z') c = (char)(c - 0x20);                    /* Read::init upper-cases */
            char cc = c == 'A' ? 'T' : c == 'G' ? 'C' : c == 'C' ? 'G' : c == 'T' ? 'A' : c == 'N' ? 'N' : 0;
            o->data[r][0][i] = c; o->qual[r][0][i] = Q[r][i];
            o->data[r][1][N[r] - 1 - i] = cc; o->qual[r][1][N[r] - 1 - i] = Q[r][i];
            countOfNs += c == 'N';
        }
        for (int d = 0; d < 2; d++) {
            memset(o->data[r][d] + N[r], 0, 32); memset(o->qual[r][d] + N[r], 0, 32);
            for (unsigned i = 0; i < N[r]; i++) o->rev[r][d][i] = o->data[r][d][N[r] - 1 - i];
            memset(o->rev[r][d] + N[r], 0, 32);
        }
    }
    if (countOfNs > maxK) return 0;                                            /* :226-228 */
    /* phase 1: seed lookups (:259-340) */
    for (unsigned r = 0; r < 2; r++) {
        unsigned next = 0, wrap = 0, nPossible = N[r] - seedLen + 1;
        uint8_t used[(MAX_READ_LENGTH + 7) / 8 + 8];
        memset(used, 0, sizeof(used));
        int begins[2] = {1, 1};
        while (nLookups[r] < nPossible && nLookups[r] < maxSeeds && nLookups[r] < P_LOOKUP_CAP) {
            if (next >= nPossible) {
                wrap++;
                begins[0] = begins[1] = 1;
                if (wrap >= seedLen) break;
                next = wrapped_next_seed(seedLen, wrap);
            }
            while (next < nPossible && (used[next / 8] & (1 << (next % 8)))) next++;
            if (next >= nPossible) continue;
            used[next / 8] |= (uint8_t)(1 << (next % 8));
            uint64_t f = 0, rv = 0;
            int valid = 1;
            for (unsigned i = 0; i < seedLen; i++) {
                int v = base_value(o->data[r][0][next + i]);
                if (v > 3) { valid = 0; break; }
                f |= (uint64_t)v << ((seedLen - i - 1) * 2);
                rv |= (uint64_t)(v ^ 3) << (i * 2);
            }
            if (!valid) { next++; continue; }                                   /* :296-302 */
            unsigned nHits[2] = {0, 0};
            const uint32_t *hits[2] = {NULL, NULL};
            uint32_t single[2] = {0, 0};
            int comp = (int64_t)f > (int64_t)rv;
            uint64_t canon = comp ? rv : f;
            uint32_t probes = 0, novf = 0;
            const uint32_t *e = ht_lookup(ix, (uint32_t)(canon >> 32), (uint32_t)canon, &probes);
            if (e) {
                for (int side = 0; side < 2; side++) {
                    uint32_t v = (side == 0) == !comp ? e[0] : e[1];
                    if (side == 1 && f == rv) { nHits[1] = nHits[0]; hits[1] = hits[0]; single[1] = single[0]; break; }
                    fill_side(ix, v, 0, INVALID_LOC, &single[side], &nHits[side], &hits[side], &novf);
                    if (hits[side] == &single[side]) hits[side] = NULL;             /* the singleton travels by value */
                }
            }
            nLookups[r]++;
            for (int d = 0; d < 2; d++) {
                uint32_t offset = d == 0 ? next : N[r] - seedLen - next;
                if (nHits[d] < o->p.maxBigHits) {
                    total[r][d] += nHits[d];
                    hs_record(&o->hs[r][d], offset, nHits[d], hits[d], single[d], begins[d]);
                    begins[d] = 0;
                } else popular[r]++;
            }
            if ((maxSeeds - nLookups[r] + 1) * seedLen + next < nPossible)        /* :333-338 */
                next += (nPossible + next) / (maxSeeds - nLookups[r] + 1);
            else next += seedLen;
        }
    }
    const unsigned more = total[0][0] + total[0][1] > total[1][0] + total[1][1] ? 0 : 1, fewer = 1 - more;   /* :342-343 */
    static const int spDir[2][2] = {{0, 1}, {1, 0}};                             /* setPairDirection, :351 */
    /* phase 2: candidates (:357-511) */
    unsigned maxUsedList = 0;
    const uint32_t maxSp = o->p.maxSpacing;
    for (unsigned sp = 0; sp < 2; sp++) {
        PHitSet *set[2];
        set[0] = &o->hs[0][sp == 0 ? 0 : 1];
        set[1] = &o->hs[1][sp == 0 ? 1 : 0];
        uint32_t fewerLoc, fewerSeed, moreLoc, moreSeed = 0;
        int outOfMore = 0;
        if (!hs_first(set[fewer], &fewerLoc, &fewerSeed)) continue;
        moreLoc = INVALID_LOC;
        for (;;) {
            if (moreLoc > fewerLoc + maxSp) {
                if (!hs_next_le(set[more], fewerLoc + maxSp, &moreLoc, &moreSeed)) break;
            }
            if (moreLoc + maxSp < fewerLoc &&
                (nMate[sp] == 0 || !is_within(o->mate[sp][nMate[sp] - 1].loc, fewerLoc, maxSp))) {
                if (!hs_next_le(set[fewer], moreLoc + maxSp, &fewerLoc, &fewerSeed)) break;
                continue;
            }
            while (moreLoc + maxSp >= fewerLoc && !outOfMore) {
                unsigned bps = hs_best_possible(set[more]);
                if (nMate[sp] >= o->poolSize / 2) { res->flags |= SNAPGPU_PFLAG_POOL_EXHAUSTED; return -1; }
                PMate *m = &o->mate[sp][nMate[sp]++];
                m->loc = moreLoc; m->bestPossible = bps; m->seedOffset = moreSeed;
                m->score = 0xfffffffeu; m->scoreLimit = 0xffffffffu; m->prob = 0; m->genomeOffset = 0;
                if (!hs_next_lower(set[more], &moreLoc, &moreSeed)) { moreLoc = 0; outOfMore = 1; break; }
            }
            unsigned bpsFewer = hs_best_possible(set[fewer]);
            unsigned lowestMate = maxK + extra;
            for (int i = (int)nMate[sp] - 1; i >= 0; i--) {
                if (o->mate[sp][i].loc > fewerLoc + maxSp) break;
                if (o->mate[sp][i].bestPossible < lowestMate) lowestMate = o->mate[sp][i].bestPossible;
            }
            if (lowestMate + bpsFewer <= maxK + extra) {
                if (nCand >= o->poolSize) { res->flags |= SNAPGPU_PFLAG_POOL_EXHAUSTED; return -1; }
                unsigned li = lowestMate + bpsFewer;
                PCand *c = &o->cand[nCand];
                c->loc = fewerLoc; c->setPair = sp; c->mateIndex = nMate[sp] - 1; c->seedOffset = fewerSeed;
                c->bestPossible = bpsFewer; c->next = o->lists[li]; c->anchor = -1;
                o->lists[li] = (int)nCand;
                nCand++;
                if (li > maxUsedList) maxUsedList = li;
            }
            if (!hs_next_lower(set[fewer], &fewerLoc, &fewerSeed)) break;
        }
    }
    /* phase 3: score and merge (:516-718) */
    double pBest = 0, pAll = 0;
    unsigned bestPairScore = 65536, scoreLimit = maxK + extra, list = 0;
    uint32_t bestLoc[2] = {0, 0}, bestScore[2] = {0, 0};
    int bestDir[2] = {0, 0};
    const uint32_t minSp = o->p.minSpacing;
    while (list <= maxUsedList && list <= scoreLimit) {
        if (o->lists[list] < 0) { list++; continue; }
        const int ci = o->lists[list];
        PCand *c = &o->cand[ci];
        uint32_t fewerScore;
        double fewerProb = 0;
        int fewerOff = 0;
        p_score_location(o, fewer, spDir[c->setPair][fewer], c->loc, c->seedOffset, scoreLimit, &fewerScore, &fewerProb,
                         &fewerOff);
        if (fewerScore != 0xffffffffu) {
            unsigned mi = c->mateIndex;
            for (;;) {
                PMate *m = &o->mate[c->setPair][mi];
                if (!is_within(m->loc, c->loc, minSp) && m->bestPossible <= scoreLimit - fewerScore) {
                    if (m->score == 0xfffffffeu || (m->score == 0xffffffffu && m->scoreLimit < scoreLimit - fewerScore)) {
                        p_score_location(o, more, spDir[c->setPair][more], m->loc, m->seedOffset, scoreLimit - fewerScore,
                                         &m->score, &m->prob, &m->genomeOffset);
                        m->scoreLimit = scoreLimit - fewerScore;
                    }
                    if (m->score != 0xffffffffu) {
                        double pairProb = m->prob * fewerProb;
                        unsigned pairScore = m->score + fewerScore;
                        int an = c->anchor;
                        const uint32_t fewerAt = c->loc + (uint32_t)fewerOff, moreAt = m->loc + (uint32_t)m->genomeOffset;
                        if (an < 0) {   /* :602-626, including the second loop's decrement */
                            for (int j = ci - 1; j >= 0 && is_within(o->cand[j].loc, fewerAt, 50) &&
                                                 o->cand[j].setPair == c->setPair; j--)
                                if (o->cand[j].anchor >= 0) { c->anchor = an = o->cand[j].anchor; break; }
                            if (an < 0)
                                for (int j = ci + 1; j >= 0 && j < (int)nCand && is_within(o->cand[j].loc, fewerAt, 50) &&
                                                     o->cand[j].setPair == c->setPair; j--)
                                    if (o->cand[j].anchor >= 0) { c->anchor = an = o->cand[j].anchor; break; }
                        }
                        int merged;
                        double oldProb;
                        if (an < 0) {
                            if (nAnchor >= o->poolSize) { res->flags |= SNAPGPU_PFLAG_POOL_EXHAUSTED; return -1; }
                            an = (int)nAnchor++;
                            PAnchor *a = &o->anchor[an];
                            a->moreLoc = moreAt; a->fewerLoc = fewerAt; a->prob = pairProb; a->pairScore = (int)pairScore;
                            merged = 0; oldProb = 0; c->anchor = an;
                        } else {   /* checkMerge, :1324-1371 */
                            PAnchor *a = &o->anchor[an];
                            if (a->moreLoc == INVALID_LOC || !(loc_distance(a->moreLoc, moreAt) < 50 && loc_distance(a->fewerLoc, fewerAt) < 50)) {
                                a->moreLoc = moreAt; a->fewerLoc = fewerAt; a->prob = pairProb; a->pairScore = (int)pairScore;
                                oldProb = 0; merged = 0;
                            } else if ((int)pairScore < a->pairScore || ((int)pairScore == a->pairScore && pairProb > a->prob)) {
                                oldProb = a->prob; a->prob = pairProb; a->pairScore = (int)pairScore; merged = 0;
                            } else { merged = 1; oldProb = 0; }
                        }
                        if (!merged) {
                            pAll = pAll - oldProb > 0 ? pAll - oldProb : 0;   /* __max(0, .) */
                            if (pairScore <= maxK && (pairScore < bestPairScore || (pairScore == bestPairScore && pairProb > pBest))) {
                                bestPairScore = pairScore;
                                pBest = pairProb;
                                bestLoc[fewer] = fewerAt; bestLoc[more] = moreAt;
                                bestScore[fewer] = fewerScore; bestScore[more] = m->score;
                                bestDir[fewer] = spDir[c->setPair][fewer]; bestDir[more] = spDir[c->setPair][more];
                                scoreLimit = bestPairScore + extra;
                            }
                            pAll += pairProb;
                            if (pAll >= 4.9) goto done;
                        }
                    }
                }
                if (mi == 0 || !is_within(o->mate[c->setPair][mi - 1].loc, c->loc, maxSp)) break;
                mi--;
            }
        }
        o->lists[list] = c->next;
    }
done:
    res->probabilityOfAllPairs = pAll;
    res->probabilityOfBestPair = pBest;
    res->popularSeedsSkipped = popular[0] + popular[1];
    if (bestPairScore == 65536) {
        for (int r = 0; r < 2; r++) { res->location[r] = INVALID_LOC; res->mapq[r] = 0; res->score[r] = -1; res->status[r] = SNAPGPU_NOT_FOUND; }
    } else {
        for (int r = 0; r < 2; r++) {
            res->location[r] = bestLoc[r];
            res->direction[r] = (uint8_t)bestDir[r];
            res->mapq[r] = oracle_compute_mapq(pAll, pBest, (int)bestScore[r], (int)(popular[0] + popular[1]));
            res->status[r] = res->mapq[r] > 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
            res->score[r] = (int)bestScore[r];
        }
    }
    return 0;
}

/* ChimericPairedEndAligner::align (:56-126) */
static int p_chimeric(POracle *o, const char *b0, const char *q0, unsigned n0, const char *b1, const char *q1, unsigned n1,
                      snapgpu_pair_result_t *res) {
    res->status[0] = res->status[1] = SNAPGPU_NOT_FOUND;
    if (n0 < 50 && n1 < 50) return 0;
    if (p_align(o, b0, q0, n0, b1, q1, n1, res)) return -1;
    res->nLocationsScored = o->nScored;
    res->fromAlignTogether = 1;
    res->alignedAsPair = 1;
    if (o->p.forceSpacing) {
        if (res->status[0] == SNAPGPU_NOT_FOUND) res->fromAlignTogether = 0;
        return 0;
    }
    if (res->status[0] != SNAPGPU_NOT_FOUND && res->status[1] != SNAPGPU_NOT_FOUND) return 0;
    const char *B[2] = {b0, b1}, *Q[2] = {q0, q1};
    unsigned N[2] = {n0, n1};
    for (int r = 0; r < 2; r++) {
        snapgpu_result_t one;
        align_read(o->single, B[r], Q[r], N[r], &one, NULL, NULL, NULL);
        if (one.flags & SNAPGPU_FLAG_READ_TOO_LONG) { res->flags |= SNAPGPU_PFLAG_READ_TOO_LONG; return -1; }
        res->status[r] = one.result;
        res->location[r] = one.location;
        res->direction[r] = one.direction;
        res->score[r] = one.score;
        res->mapq[r] = one.mapq / 4;
        res->nSingleScored += one.nLocationsScored;
    }
    res->fromAlignTogether = 0;
    res->alignedAsPair = 0;
    return 0;
}

static snapgpu_aligner_params_t p_single_params(const snapgpu_paired_params_t *p) {
    snapgpu_aligner_params_t a;
    memset(&a, 0, sizeof(a));
    a.maxHitsToConsider = p->maxHits; a.maxK = p->maxK; a.maxReadSize = p->maxReadSize;
    a.maxSeedsToUse = p->maxSeedsToUse; a.maxSeedCoverage = p->seedCoverage; a.extraSearchDepth = p->extraSearchDepth;
    return a;
}

typedef struct {
    const snapgpu_index_view_t *ix;
    const snapgpu_paired_params_t *p;
    const char *b0, *q0, *b1, *q1;
    const uint64_t *o0, *o1;
    const uint32_t *l0, *l1;
    uint64_t n;
    int chimeric;
    snapgpu_pair_result_t *out;
    volatile uint64_t *cursor;
} PJob;

static void *p_worker(void *arg) {
    PJob *j = (PJob *)arg;
    POracle *o = (POracle *)calloc(1, sizeof(POracle));
    o->ix = j->ix;
    o->p = *j->p;
    o->maxSeedsCmd = j->p->maxSeedsToUse < P_MAX_SEEDS ? j->p->maxSeedsToUse : P_MAX_SEEDS;   /* __min(MAX_MAX_SEEDS, .) :47 */
    unsigned maxSeedsToUse = o->maxSeedsCmd ? o->maxSeedsCmd
                                            : (unsigned)(j->p->maxReadSize * j->p->seedCoverage / j->ix->seedLen);
    uint64_t pool = (uint64_t)j->p->maxBigHits * maxSeedsToUse * 2;                         /* :128 */
    o->poolSize = (unsigned)(pool < j->p->maxCandidatePoolSize ? pool : j->p->maxCandidatePoolSize);
    o->cand = (PCand *)calloc(o->poolSize + 1, sizeof(PCand));
    o->mate[0] = (PMate *)calloc(o->poolSize / 2 + 1, sizeof(PMate));
    o->mate[1] = (PMate *)calloc(o->poolSize / 2 + 1, sizeof(PMate));
    o->anchor = (PAnchor *)calloc(o->poolSize + 1, sizeof(PAnchor));
    o->lists = (int *)calloc(j->p->maxK + j->p->extraSearchDepth + 2, sizeof(int));
    snapgpu_aligner_params_t sp = p_single_params(j->p);
    if (j->chimeric) o->single = oracle_new(j->ix, &sp, 0);
    for (;;) {
        uint64_t b = __atomic_fetch_add(j->cursor, 16, __ATOMIC_RELAXED);
        if (b >= j->n) break;
        uint64_t e = b + 16 < j->n ? b + 16 : j->n;
        for (uint64_t i = b; i < e; i++) {
            snapgpu_pair_result_t *r = &j->out[i];
            pair_pre(r);
            const char *B0 = j->b0 + j->o0[i], *Q0 = j->q0 + j->o0[i], *B1 = j->b1 + j->o1[i], *Q1 = j->q1 + j->o1[i];
            if (j->chimeric) p_chimeric(o, B0, Q0, j->l0[i], B1, Q1, j->l1[i], r);
            else { p_align(o, B0, Q0, j->l0[i], B1, Q1, j->l1[i], r); r->nLocationsScored = o->nScored; }
        }
    }
    if (o->single) oracle_delete(o->single);
    free(o->cand); free(o->mate[0]); free(o->mate[1]); free(o->anchor); free(o->lists); free(o);
    return NULL;
}

/* Pairs (reads0[i], reads1[i]); chimeric = 1: ChimericPairedEndAligner::align, 0: the
 * IntersectingPairedEndAligner alone. */
int oracle_paired_batch(const snapgpu_index_view_t *ix, const snapgpu_paired_params_t *p, const char *b0, const char *q0,
                        const uint64_t *o0, const uint32_t *l0, const char *b1, const char *q1, const uint64_t *o1,
                        const uint32_t *l1, uint64_t n, int chimeric, snapgpu_pair_result_t *out, int nThreads) {
    if (ix->seedLen < 16 || ix->seedLen > 25) return -1;
    pthread_once(&g_once, init_tables);
    if (nThreads < 1) nThreads = 1;
    volatile uint64_t cursor = 0;
    PJob job = {ix, p, b0, q0, b1, q1, o0, o1, l0, l1, n, chimeric, out, &cursor};
    pthread_t *th = (pthread_t *)calloc((size_t)nThreads, sizeof(pthread_t));
    for (int t = 0; t < nThreads; t++) pthread_create(&th[t], NULL, p_worker, &job);
    for (int t = 0; t < nThreads; t++) pthread_join(th[t], NULL);
    free(th);
    return 0;
}

/* ================================================================ CharacterizeSeeds
 * BaseAligner::CharacterizeSeeds (BaseAligner.cpp:206-508) as the partial aligner of
 * PairedAligner.cpp:518-527 runs it: AlignRead's seed order, unwindowed lookups, every hit of a
 * non-popular side recorded under (direction, hit - offset) with the seed offset `next`.  The
 * two std::map<unsigned, std::set<unsigned>> are rebuilt as sorted (dir, location, offset)
 * keys reduced to runs {location, *set.begin(), *set.rbegin(), set.size()} -- map order: map,
 * then mapRC, locations ascending.  Test infrastructure (pinned to ref_harness_rna charseeds). */
static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

int oracle_characterize_seeds(const snapgpu_index_view_t *ix, unsigned maxHits, unsigned maxK, unsigned numSeeds,
                              int explore, const char *bases, const uint64_t *offsets, const uint32_t *lengths,
                              uint64_t n, uint64_t *start, uint32_t *nForward, snapgpu_seed_run_t *runs, uint64_t cap) {
    const unsigned seedLen = ix->seedLen;
    uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)(numSeeds + 2) * maxHits + 64));
    if (!keys) return -1;
    uint64_t at = 0;
    for (uint64_t r = 0; r < n; r++) {
        start[r] = at;
        nForward[r] = 0;
        const unsigned len = lengths[r];
        const char *b = bases + offsets[r];
        if (len > 500 || len < seedLen) continue;   /* :272-282 (too long: the reference exits) */
        char fwd[512 + 32];
        unsigned nN = 0;
        for (unsigned i = 0; i < len; i++) {
            char c = b[i];
            if (c >= 'a' && c <= 'z') c = (char)(c - 0x20);
            fwd[i] = c;
            nN += c == 'N';
        }
        if (nN > maxK) continue;   /* :303-306 */
        uint8_t used[64];
        memset(used, 0, sizeof(used));
        unsigned nPossible = len - seedLen + 1, next = 0, wrapCount = 0, applied[2] = {0, 0};
        size_t nk = 0;
        while (applied[0] + applied[1] < numSeeds) {   /* :336 */
            if (next >= nPossible) {
                wrapCount++;
                if (wrapCount >= seedLen) break;   /* :348-354 */
                next = wrapped_next_seed(seedLen, wrapCount);
            }
            while (next < nPossible && (used[next / 8] & (1 << (next % 8)))) next++;
            if (next >= nPossible) continue;
            used[next / 8] |= (uint8_t)(1 << (next % 8));
            uint64_t f = 0, rr = 0;
            int valid = 1;
            for (unsigned i = 0; i < seedLen; i++) {
                int v = base_value(fwd[next + i]);
                if (v > 3) { valid = 0; break; }
                f |= (uint64_t)v << ((seedLen - i - 1) * 2);
                rr |= (uint64_t)(v ^ 3) << (i * 2);
            }
            if (!valid) continue;   /* :375-377 */
            unsigned nHits[2] = {0, 0}, nOvf = 0;
            const uint32_t *hits[2] = {NULL, NULL};
            uint32_t singleton[2], probes = 0;
            int comp = (int64_t)f > (int64_t)rr;
            uint64_t canon = comp ? rr : f;
            const uint32_t *e = ht_lookup(ix, (uint32_t)(canon >> 32), (uint32_t)canon, &probes);
            if (e) {
                for (int side = 0; side < 2; side++) {
                    uint32_t v = (side == 0) == !comp ? e[0] : e[1];
                    if (side == 1 && f == rr) { nHits[1] = nHits[0]; hits[1] = hits[0]; break; }
                    fill_side(ix, v, 0, INVALID_LOC, &singleton[side], &nHits[side], &hits[side], &nOvf);
                }
            }
            for (int dir = 0; dir < 2; dir++) {   /* :393-497 */
                if (nHits[dir] > maxHits && !explore) continue;
                const unsigned offset = dir == 0 ? next : len - seedLen - next;
                const unsigned lim = nHits[dir] < maxHits ? nHits[dir] : maxHits;
                for (unsigned i = 0; i < lim; i++) {
                    const uint32_t h = hits[dir][i];
                    if (h < offset) continue;
                    keys[nk++] = ((uint64_t)dir << 41) | ((uint64_t)(h - offset) << 9) | next;
                }
                applied[dir]++;
            }
            next += seedLen;
        }
        qsort(keys, nk, sizeof(uint64_t), cmp_u64);
        for (size_t i = 0; i < nk;) {
            size_t j = i;
            while (j + 1 < nk && (keys[j + 1] >> 9) == (keys[i] >> 9)) j++;
            if (at >= cap) { free(keys); return -2; }
            snapgpu_seed_run_t *o = &runs[at++];
            o->location = (uint32_t)(keys[i] >> 9);
            o->minOffset = (uint16_t)(keys[i] & 511);
            o->maxOffset = (uint16_t)(keys[j] & 511);
            o->count = (uint16_t)(j - i + 1);
            o->direction = (uint8_t)(keys[i] >> 41);
            o->reserved = 0;
            if (!o->direction) nForward[r]++;
            i = j + 1;
        }
    }
    start[n] = at;
    free(keys);
    return 0;
}

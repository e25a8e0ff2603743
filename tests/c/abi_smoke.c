/* A plain-C caller of the C ABI (include/snapgpu.h), compiled and run by tests/test_capi.py
 * (CPU) and tests/test_capi.py::test_plain_c_caller_aligns_on_gpu (GPU): the header is valid C99
 * and the entry points behave as declared, called the way a SNAPLib-side binding would call them
 * (Aligner.h:54-80: one batched AlignRead over a read buffer).
 *
 *   abi_smoke            host-side entry points; without a GPU snapgpu_aligner_create must fail
 *                        loudly (NULL + error message) -- there is no CPU fallback
 *   abi_smoke N          ... and, when a device exists, N synthetic 100-bp reads aligned through
 *                        snapgpu_align_batch, one canonical record per read on stdout:
 *                        "R <i> <result> <location> <direction> <score> <mapq> <nLookups>
 *                         <nLocationsScored> <popularSeedsSkipped> <nHitsIgnored> <nHitWords>
 *                         <nOverflowLists> <nElements> <pAll bits> <pBest bits>"
 *                        (every field the parity tests compare; nProbes is a device statistic)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "snapgpu.h"

static unsigned long long bits(double d) {
    unsigned long long u;
    memcpy(&u, &d, sizeof u);
    return u;
}

int main(int argc, char **argv) {
    const unsigned long nReads = argc > 1 ? strtoul(argv[1], NULL, 10) : 0;
    snapgpu_synth_genome_params_t gp;
    memset(&gp, 0, sizeof gp);
    gp.seed = 7; gp.totalBases = 200000; gp.nContigs = 2; gp.nRepeatFamilies = 10;
    gp.repeatFraction = 0.3; gp.maxDivergence = 0.1; gp.nRunFraction = 0.001; gp.chromosomePadding = 500;
    snapgpu_genome_t *g = snapgpu_genome_synthetic(&gp);
    if (!g) { printf("genome: %s\n", snapgpu_last_error()); return 1; }
    char seed[21];
    memcpy(seed, snapgpu_genome_bases(g) + snapgpu_genome_piece_offset(g, 0) + 1000, 20);
    seed[20] = 0;
    snapgpu_index_t *idx = snapgpu_index_build(g, 20, 2);   /* takes ownership of g */
    if (!idx) { printf("index: %s\n", snapgpu_last_error()); return 1; }
    snapgpu_index_info_t info;
    if (snapgpu_index_get_info(idx, &info) != 0 || info.seedLen != 20) { printf("info\n"); return 1; }
    uint32_t n[2], f[64], r[64];
    int ok = 1;
    if (strchr(seed, 'N') == NULL && strchr(seed, 'n') == NULL) {
        if (snapgpu_index_lookup(idx, seed, n, f, r, 64) != 0) { printf("lookup: %s\n", snapgpu_last_error()); return 1; }
        ok = n[0] + n[1] >= 1;   /* the seed occurs where it was taken from */
    }
    snapgpu_aligner_params_t p;
    snapgpu_aligner_params_default(&p);
    snapgpu_aligner_t *a = snapgpu_aligner_create(0, idx, &p);
    int gpus = snapgpu_device_count();
    if (gpus == 0 && a != NULL) { printf("aligner created without a GPU\n"); return 1; }
    if (!a) printf("aligner_create: %s\n", snapgpu_last_error());
    unsigned long aligned = 0, single = 0;
    if (a && nReads > 0) {
        snapgpu_synth_reads_params_t rp;
        memset(&rp, 0, sizeof rp);
        rp.seed = 31; rp.nReads = nReads; rp.readLength = 100; rp.qualityChar = '2';
        rp.baseErrorRate = 0.02; rp.mutationRate = 0.001; rp.indelFraction = 0.15; rp.indelExtend = 0.3;
        rp.randomReadFraction = 0.02;
        snapgpu_reads_t *reads = snapgpu_reads_synthetic(snapgpu_index_genome(idx), &rp);
        snapgpu_result_t *out = reads ? (snapgpu_result_t *)calloc(nReads, sizeof *out) : NULL;
        if (!reads || !out) { printf("reads: %s\n", snapgpu_last_error()); return 1; }
        if (snapgpu_align_batch(a, reads, out) != SNAPGPU_OK) { printf("align: %s\n", snapgpu_last_error()); return 1; }
        for (unsigned long i = 0; i < nReads; i++) {
            const snapgpu_result_t *o = &out[i];
            printf("R %lu %u %u %u %d %d %u %u %u %u %u %u %u %016llx %016llx\n", i, o->result, o->location,
                   o->direction, o->score, o->mapq, o->nLookups, o->nLocationsScored, o->popularSeedsSkipped,
                   o->nHitsIgnored, o->nHitWords, o->nOverflowLists, o->nElements,
                   bits(o->probabilityOfAllCandidates), bits(o->probabilityOfBestCandidate));
            single += o->result == SNAPGPU_SINGLE_HIT;
        }
        aligned = nReads;
        free(out);
        snapgpu_reads_free(reads);
    }
    if (a) snapgpu_aligner_free(a);
    snapgpu_index_free(idx);
    printf("ok %d gpus %d aligned %lu single %lu\n", ok, gpus, aligned, single);
    return ok ? 0 : 1;
}

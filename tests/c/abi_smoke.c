/* A plain-C caller of the C ABI (include/snapgpu.h), compiled and run by
 * tests/test_capi.py: the header is valid C99 and the host-side entry points behave
 * as declared.  Without a GPU, snapgpu_aligner_create must fail loudly (NULL + error
 * message) -- there is no CPU fallback. */
#include <stdio.h>
#include <string.h>

#include "snapgpu.h"

int main(void) {
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
    if (a) snapgpu_aligner_free(a);
    else printf("aligner_create: %s\n", snapgpu_last_error());
    snapgpu_index_free(idx);
    printf("ok %d gpus %d\n", ok, gpus);
    return ok ? 0 : 1;
}

// GpuPairedEndAligner.cpp -- see GpuPairedEndAligner.h.  C++98, SNAPLib headers.
#include "GpuPairedEndAligner.h"

#include "exit.h"

#include <vector>

static void pairedFail(const char *what) {
    fprintf(stderr, "MI355X paired aligner: %s: %s\n", what, snapgpu_last_error());
    soft_exit(1);
}

GpuPairedEndAligner::GpuPairedEndAligner(const char *indexDir, int device, unsigned maxReadSize, unsigned maxHits,
                                         unsigned maxK, unsigned numSeeds, double seedCoverage, unsigned minSpacing,
                                         unsigned maxSpacing, unsigned maxBigHits, unsigned extraSearchDepth,
                                         unsigned maxCandidatePoolSize, bool forceSpacing)
    : idx(NULL), gpu(NULL), locationsScored(0), nPerPair(0)
{
    idx = snapgpu_index_load(indexDir);
    if (idx == NULL) pairedFail("index load");
    snapgpu_paired_params_t p;
    snapgpu_paired_params_default(&p);
    p.maxHits = maxHits;
    p.maxK = maxK;
    p.maxSeedsToUse = numSeeds;
    p.seedCoverage = seedCoverage;
    p.minSpacing = minSpacing;
    p.maxSpacing = maxSpacing;
    p.maxBigHits = maxBigHits;
    p.extraSearchDepth = extraSearchDepth;
    p.maxCandidatePoolSize = maxCandidatePoolSize;
    p.maxReadSize = maxReadSize;
    p.forceSpacing = forceSpacing ? 1 : 0;
    gpu = snapgpu_paired_aligner_create(device, idx, &p);   // no GPU: fails here, loudly
    if (gpu == NULL) pairedFail("aligner create");
}

GpuPairedEndAligner::~GpuPairedEndAligner()
{
    snapgpu_paired_aligner_free(gpu);
    snapgpu_index_free(idx);
}

void GpuPairedEndAligner::align(Read *read0, Read *read1, PairedAlignmentResult *result)
{
    if (nPerPair++ == 0)
        fprintf(stderr, "MI355X paired aligner: align() aligns one pair per GPU batch (copy in, the passes, copy out); "
                        "batch the caller through GpuPairedEndAligner::alignBatch\n");
    alignBatch(&read0, &read1, 1, result);
}

void GpuPairedEndAligner::alignBatch(Read **reads0, Read **reads1, unsigned n, PairedAlignmentResult *results)
{
    if (n == 0) return;
    Read **R[2] = {reads0, reads1};
    snapgpu_reads_t *batch[2] = {NULL, NULL};
    for (int e = 0; e < 2; e++) {
        std::vector<char> b, q;
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n);
        for (unsigned i = 0; i < n; i++) {
            off[i] = b.size();
            len[i] = R[e][i]->getDataLength();
            b.insert(b.end(), R[e][i]->getData(), R[e][i]->getData() + len[i]);
            q.insert(q.end(), R[e][i]->getQuality(), R[e][i]->getQuality() + len[i]);
        }
        b.push_back(0);
        q.push_back(0);
        batch[e] = snapgpu_reads_from_arrays(n, &b[0], &q[0], &off[0], &len[0]);
        if (batch[e] == NULL) pairedFail("read copy");
    }
    std::vector<snapgpu_pair_result_t> out(n);
    const int rc = snapgpu_paired_align_batch(gpu, batch[0], batch[1], &out[0]);
    snapgpu_reads_free(batch[0]);
    snapgpu_reads_free(batch[1]);
    if (rc != SNAPGPU_OK) pairedFail("align");   // includes the reference's own soft_exit cases
    for (unsigned i = 0; i < n; i++) {
        PairedAlignmentResult &r = results[i];
        const snapgpu_pair_result_t &o = out[i];
        for (int k = 0; k < NUM_READS_PER_PAIR; k++) {
            r.status[k] = (AlignmentResult)o.status[k];
            r.location[k] = o.location[k];
            r.direction[k] = (Direction)o.direction[k];
            r.score[k] = o.score[k];
            r.mapq[k] = o.mapq[k];
            r.isTranscriptome[k] = false;
            r.tlocation[k] = 0;
        }
        r.fromAlignTogether = o.fromAlignTogether != 0;
        r.alignedAsPair = o.alignedAsPair != 0;
        r.nanosInAlignTogether = 0;
        r.nLVCalls = 0;
        r.nSmallHits = 0;
        locationsScored += o.nLocationsScored + o.nSingleScored;
    }
}

_int64 GpuPairedEndAligner::getLocationsScored() const { return locationsScored; }

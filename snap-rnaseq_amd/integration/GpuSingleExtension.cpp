// GpuSingleExtension.cpp -- see GpuSingleExtension.h.  C++98, SNAPLib headers.
#include "GpuSingleExtension.h"
#include "multihit_copy.h"

#include "AlignmentFilter.h"
#include "GenomeIndex.h"
#include "exit.h"

#include <string>
#include <vector>

static void gpuFail(const char *what) {
    fprintf(stderr, "MI355X aligner: %s: %s\n", what, snapgpu_last_error());
    soft_exit(1);
}

// ------------------------------------------------------------------ GpuBaseAligner
GpuBaseAligner::GpuBaseAligner(const char *indexDir, int device, unsigned maxHits, unsigned maxK,
                               unsigned maxReadSize, unsigned numSeeds, double seedCoverage,
                               unsigned extraSearchDepth, bool explorePopular, bool stopOnFirst)
    : idx(NULL), gpu(NULL), ignoredReads(0), nPerRead(0)
{
    idx = snapgpu_index_load(indexDir);
    if (idx == NULL) gpuFail("index load");
    snapgpu_aligner_params_t p;
    snapgpu_aligner_params_default(&p);
    p.maxHitsToConsider = maxHits;
    p.maxK = maxK;
    p.maxReadSize = maxReadSize;
    p.maxSeedsToUse = numSeeds;
    p.maxSeedCoverage = seedCoverage;
    p.extraSearchDepth = extraSearchDepth;
    p.explorePopularSeeds = explorePopular ? 1 : 0;
    p.stopOnFirstHit = stopOnFirst ? 1 : 0;
    gpu = snapgpu_aligner_create(device, idx, &p);   // no GPU: fails here, loudly
    if (gpu == NULL) gpuFail("aligner create");
}

GpuBaseAligner::~GpuBaseAligner()
{
    snapgpu_aligner_free(gpu);
    snapgpu_index_free(idx);
}

// The reads copied into one batch (a Read is only valid until the next getNextRead, Read.h:135)
snapgpu_reads_t *GpuBaseAligner::copyReads(Read **reads, unsigned n)
{
    std::vector<char> b, q;
    std::vector<uint64_t> off(n + 1);
    std::vector<uint32_t> len(n + 1);
    for (unsigned i = 0; i < n; i++) {
        off[i] = b.size();
        len[i] = reads[i]->getDataLength();
        b.insert(b.end(), reads[i]->getData(), reads[i]->getData() + len[i]);
        q.insert(q.end(), reads[i]->getQuality(), reads[i]->getQuality() + len[i]);
    }
    b.push_back(0);
    q.push_back(0);
    snapgpu_reads_t *r = snapgpu_reads_from_arrays(n, &b[0], &q[0], &off[0], &len[0]);
    if (r == NULL) gpuFail("read copy");
    return r;
}

static void tooLong(const snapgpu_result_t &o)
{
    if (o.flags & SNAPGPU_FLAG_READ_TOO_LONG) {   // BaseAligner.cpp:609-613
        fprintf(stderr, "Read is too long\n");
        soft_exit(1);
    }
}

AlignmentResult GpuBaseAligner::AlignRead(Read *read, unsigned *genomeLocation, Direction *hitDirection,
                                          int *finalScore, int *mapq)
{
    if (nPerRead++ == 0)
        fprintf(stderr, "MI355X aligner: AlignRead aligns one read per GPU batch (copy in, the passes, copy out); "
                        "batch the caller through GpuBaseAligner::AlignReads / AlignReadsMultiHit\n");
    AlignmentResult r;
    int s = 0, q = 0;
    AlignReads(&read, 1, &r, genomeLocation, hitDirection, &s, &q);
    if (finalScore != NULL) *finalScore = s;
    if (mapq != NULL) *mapq = q;
    return r;
}

void GpuBaseAligner::AlignReads(Read **reads, unsigned n, AlignmentResult *results, unsigned *genomeLocations,
                                Direction *hitDirections, int *finalScores, int *mapqs)
{
    if (n == 0) return;
    snapgpu_reads_t *r = copyReads(reads, n);
    std::vector<snapgpu_result_t> o(n);
    const int rc = snapgpu_align_batch(gpu, r, &o[0]);
    snapgpu_reads_free(r);
    if (rc != SNAPGPU_OK) gpuFail("align");
    for (unsigned i = 0; i < n; i++) {
        tooLong(o[i]);
        results[i] = (AlignmentResult)o[i].result;
        genomeLocations[i] = o[i].location;
        hitDirections[i] = (Direction)o[i].direction;
        if (finalScores != NULL) finalScores[i] = o[i].score;
        if (mapqs != NULL) mapqs[i] = o[i].mapq;
    }
}

void GpuBaseAligner::AlignReadsMultiHit(Read **reads, unsigned n, unsigned maxHitsToGet, AlignmentResult *results,
                                        unsigned *genomeLocations, Direction *hitDirections, int *finalScores,
                                        int *mapqs, int *multiHitsFound, unsigned *multiHitLocations,
                                        bool *multiHitRCs, int *multiHitScores)
{
    if (n == 0) return;
    snapgpu_reads_t *r = copyReads(reads, n);
    std::vector<snapgpu_result_t> o(n);
    std::vector<snapgpu_multi_hit_t> h((size_t)n * (maxHitsToGet > 0 ? maxHitsToGet : 1));
    const int rc = snapgpu_align_batch_ex(gpu, r, NULL, maxHitsToGet, &o[0], multiHitsFound, &h[0]);
    snapgpu_reads_free(r);
    if (rc != SNAPGPU_OK) gpuFail("align (multi-hit)");
    for (unsigned i = 0; i < n; i++) {
        tooLong(o[i]);
        results[i] = (AlignmentResult)o[i].result;
        genomeLocations[i] = o[i].location;
        hitDirections[i] = (Direction)o[i].direction;
        if (finalScores != NULL) finalScores[i] = o[i].score;
        if (mapqs != NULL) mapqs[i] = o[i].mapq;
        // nothing when maxHitsToGet == 0 (multiHitsFound is then not written), else at most a row
        gpuCopyMultiHits(&h[0], i, maxHitsToGet, maxHitsToGet ? multiHitsFound[i] : 0, multiHitLocations,
                         multiHitRCs, multiHitScores);
    }
}

snapgpu_aligner_stats_t GpuBaseAligner::stats() const
{
    snapgpu_aligner_stats_t s;
    snapgpu_aligner_get_stats(gpu, &s);
    return s;
}
_int64 GpuBaseAligner::getNHashTableLookups() const { return stats().nHashTableLookups; }
_int64 GpuBaseAligner::getLocationsScored() const { return stats().nLocationsScored; }
_int64 GpuBaseAligner::getNHitsIgnoredBecauseOfTooHighPopularity() const
{
    return stats().nHitsIgnoredBecauseOfTooHighPopularity;
}
_int64 GpuBaseAligner::getNReadsIgnoredBecauseOfTooManyNs() const
{
    return stats().nReadsIgnoredBecauseOfTooManyNs + ignoredReads;
}
_int64 GpuBaseAligner::getNIndelsMerged() const { return stats().nIndelsMerged; }
void GpuBaseAligner::addIgnoredReads(_int64 n) { ignoredReads += n; }
const char *GpuBaseAligner::getRCTranslationTable() const { return NULL; }
int GpuBaseAligner::getMaxK() const { return snapgpu_aligner_max_k(gpu); }
const char *GpuBaseAligner::getName() const { return snapgpu_aligner_name(gpu); }

// -------------------------------------------------------------- GpuSingleExtension
struct GpuSingleExtension::Shared {
    snapgpu_index_t *genome, *transcriptome;
    snapgpu_aligner_params_t params;
    int nextDevice;
    ExclusiveLock lock;
};

GpuSingleExtension::GpuSingleExtension(unsigned batch, int dev)
    : shared(NULL), owner(true), batchReads(batch), device(dev), g(NULL), t(NULL)
{
}

GpuSingleExtension::GpuSingleExtension(Shared *s, unsigned batch, int dev)
    : shared(s), owner(false), batchReads(batch), device(dev), g(NULL), t(NULL)
{
}

GpuSingleExtension::~GpuSingleExtension()
{
    finishThread();
    if (owner && shared != NULL) {
        snapgpu_index_free(shared->genome);
        snapgpu_index_free(shared->transcriptome);
        DestroyExclusiveLock(&shared->lock);
        delete shared;
    }
}

void GpuSingleExtension::initialize()
{
    // AlignerContext::runAlignment calls this once, before options are parsed into the context;
    // the index directories come from the command line the context parses later, so the
    // indexes are loaded lazily by the first thread (beginThread) under the lock.
    if (shared == NULL) {
        shared = new Shared();
        shared->genome = shared->transcriptome = NULL;
        shared->nextDevice = 0;
        InitializeExclusiveLock(&shared->lock);
    }
}

AlignerExtension *GpuSingleExtension::copy()
{
    initialize();
    return new GpuSingleExtension(shared, batchReads, device);
}

void GpuSingleExtension::beginThread() {}

void GpuSingleExtension::finishThread()
{
    snapgpu_aligner_free(g);
    snapgpu_aligner_free(t);
    g = t = NULL;
}

bool GpuSingleExtension::runIterationThread(ReadSupplier *supplier, AlignerContext *ctx)
{
    AlignerOptions *options = ctx->options;
    if (ctx->contamination != NULL) {
        fprintf(stderr, "MI355X aligner: the contamination database (-x) is not supported\n");
        soft_exit(1);
    }
    if (g == NULL) {
        AcquireExclusiveLock(&shared->lock);
        if (shared->genome == NULL) {
            shared->genome = snapgpu_index_load(options->indexDir);
            shared->transcriptome = snapgpu_index_load(options->transcriptomeDir);
            if (shared->genome == NULL || shared->transcriptome == NULL) gpuFail("index load");
            // the aligners SingleAligner.cpp:165-203 constructs
            snapgpu_aligner_params_default(&shared->params);
            shared->params.maxHitsToConsider = ctx->maxHits;
            shared->params.maxK = ctx->maxDist;
            shared->params.maxReadSize = MAX_READ_LENGTH;
            shared->params.maxSeedsToUse = ctx->numSeedsFromCommandLine;
            shared->params.maxSeedCoverage = ctx->seedCoverage;
            shared->params.extraSearchDepth = ctx->extraSearchDepth;
            shared->params.explorePopularSeeds = options->explorePopularSeeds ? 1 : 0;
            shared->params.stopOnFirstHit = options->stopOnFirstHit ? 1 : 0;
        }
        const int nDev = snapgpu_device_count();
        const int dev = device >= 0 ? device : (nDev > 0 ? shared->nextDevice++ % nDev : 0);
        ReleaseExclusiveLock(&shared->lock);
        g = snapgpu_aligner_create(dev, shared->genome, &shared->params);
        if (g == NULL) gpuFail("genome aligner");
        t = snapgpu_aligner_create(dev, shared->transcriptome, &shared->params);
        if (t == NULL) gpuFail("transcriptome aligner");
    }
    // One batch at a time: copy every read (unclipped bytes + its clip and read group), align
    // the useful ones on the GPU, then the reference's per-read tail in input order.
    std::vector<char> data, qual, ids;
    std::vector<uint64_t> dOff, idOff, uOff;
    std::vector<uint32_t> uLen, front, clipped, full, idLen;
    std::vector<const char *> rg;
    std::vector<int> useful;
    for (bool more = true; more;) {
        data.clear(); qual.clear(); ids.clear(); dOff.clear(); idOff.clear(); uOff.clear(); uLen.clear();
        front.clear(); clipped.clear(); full.clear(); idLen.clear(); rg.clear(); useful.clear();
        Read *read = NULL;
        while (useful.size() < batchReads && (read = supplier->getNextRead()) != NULL) {
            ctx->stats->totalReads++;
            // pre-filter, SingleAligner.cpp:247-257
            const bool quality = read->qualityFilter(options->minPercentAbovePhred, options->minPhred,
                                                     options->phredOffset);
            const bool use = !(read->getDataLength() < 50 || read->countOfNs() > ctx->maxDist || !quality);
            if (use) ctx->stats->usefulReads++;
            dOff.push_back(data.size());
            data.insert(data.end(), read->getUnclippedData(), read->getUnclippedData() + read->getUnclippedLength());
            qual.insert(qual.end(), read->getUnclippedQuality(), read->getUnclippedQuality() + read->getUnclippedLength());
            idOff.push_back(ids.size());
            ids.insert(ids.end(), read->getId(), read->getId() + read->getIdLength());
            idLen.push_back(read->getIdLength());
            front.push_back(read->getFrontClippedLength());
            clipped.push_back(read->getDataLength());
            full.push_back(read->getUnclippedLength());
            rg.push_back(read->getReadGroup());
            useful.push_back(use ? 1 : 0);
            if (use) {
                uOff.push_back(dOff.back() + front.back());
                uLen.push_back(read->getDataLength());
            }
        }
        more = read != NULL;
        if (useful.empty()) break;
        data.resize(data.size() + 16, 0);
        ids.push_back(0);
        qual.resize(qual.size() + 16, 0);
        const size_t nu = uLen.size();
        std::vector<snapgpu_result_t> tr(nu + 1), gr(nu + 1);
        if (nu > 0) {
            snapgpu_reads_t *r = snapgpu_reads_from_arrays(nu, &data[0], &qual[0], &uOff[0], &uLen[0]);
            if (r == NULL) gpuFail("batch");
            if (snapgpu_align_batch(t, r, &tr[0]) != SNAPGPU_OK) gpuFail("transcriptome align");   // SingleAligner.cpp:270
            if (snapgpu_align_batch(g, r, &gr[0]) != SNAPGPU_OK) gpuFail("genome align");          // SingleAligner.cpp:274
            snapgpu_reads_free(r);
        }
        size_t j = 0;
        for (size_t i = 0; i < useful.size(); i++) {
            Read r;
            r.init(&ids[idOff[i]], idLen[i], &data[dOff[i]], &qual[dOff[i]], full[i]);
            r.clip(ctx->clipping);
            r.setReadGroup(rg[i]);
            if (!useful[i]) {   // SingleAligner.cpp:250-254
                if (ctx->readWriter != NULL && options->passFilter(&r, NotFound)) {
                    ctx->readWriter->writeRead(&r, NotFound, 0, InvalidGenomeLocation, false, false, 0);
                }
                continue;
            }
            unsigned location = InvalidGenomeLocation, tlocation = 0;
            Direction direction = FORWARD;
            int score = 0, mapq = 0;
            bool isTranscriptome = false;
            AlignmentFilter filter(NULL, &r, ctx->index->getGenome(), ctx->transcriptome->getGenome(), ctx->gtf, 0, 0,
                                   options->confDiff, options->maxDist.start, ctx->index->getSeedLength(), NULL);
            filter.AddAlignment(tr[j].location, (Direction)tr[j].direction, tr[j].score, tr[j].mapq, true, true);
            filter.AddAlignment(gr[j].location, (Direction)gr[j].direction, gr[j].score, gr[j].mapq, false, true);
            j++;
            AlignmentResult result = filter.FilterSingle(&location, &direction, &score, &mapq, &isTranscriptome, &tlocation);
            // SingleAlignerContext::writeRead / updateStats (SingleAligner.cpp:322-365)
            if (ctx->readWriter != NULL && options->passFilter(&r, result)) {
                ctx->readWriter->writeRead(&r, result, mapq, location, direction, isTranscriptome, tlocation);
            }
            if (isOneLocation(result)) ctx->stats->singleHits++;
            else if (result == MultipleHits) ctx->stats->multiHits++;
            else ctx->stats->notFound++;
            if (result != NotFound) ctx->stats->mapqHistogram[mapq]++;
        }
    }
    return true;
}

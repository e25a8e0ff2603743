// GpuSingleExtension.h -- the drop-in for SNAPLib: what a SNAPLib maintainer adds to run
// `snap-rna single` on MI355X GPUs.  Written against the reference's own
// headers (SNAPLib/AlignerContext.h, Aligner.h, Read.h, AlignmentFilter.h) in the reference's
// dialect (C++98); tests/test_integration_build.py compiles and links it with the reference's
// objects in the build container.
//
//  * GpuBaseAligner : Aligner -- BaseAligner::AlignRead (BaseAligner.cpp:196-200).  The Aligner
//    interface aligns one read per call, which on the GPU is a one-read batch (H2D, the passes,
//    D2H per read): it works for any existing caller of Aligner* but is slower than the CPU, and
//    says so on stderr the first time.  Batching callers use AlignReads (n reads, one batch) and
//    AlignReadsMultiHit (the richer AlignRead with multi-hit export that PairedAligner.cpp:602-605
//    calls per pair, for n reads in one batch).
//  * GpuSingleExtension : AlignerExtension -- the hook SingleAlignerContext::runIterationThread
//    calls first (SingleAligner.cpp:150-153, AlignerContext.h:157): the thread's reads are taken
//    in batches, both AlignRead calls of every read run as two GPU batches, and the unchanged
//    host tail (the reference's AlignmentFilter, ReadWriter, stats) runs per read in input order.
#pragma once

#include "stdafx.h"
#include "Aligner.h"
#include "AlignerContext.h"
#include "AlignerOptions.h"
#include "Read.h"
#include "snapgpu.h"

class GpuBaseAligner : public Aligner {
public:
    // The index is the reference's on-disk index directory (snapgpu_index_load reads it).
    GpuBaseAligner(const char *indexDir, int device, unsigned maxHits, unsigned maxK, unsigned maxReadSize,
                   unsigned numSeeds, double seedCoverage, unsigned extraSearchDepth, bool explorePopular,
                   bool stopOnFirst);
    virtual ~GpuBaseAligner();

    virtual AlignmentResult AlignRead(Read *read, unsigned *genomeLocation, Direction *hitDirection,
                                      int *finalScore = NULL, int *mapq = NULL);
    // AlignRead of reads[0..n) in one GPU batch; outputs per read as AlignRead returns them
    // (finalScores / mapqs may be NULL)
    void AlignReads(Read **reads, unsigned n, AlignmentResult *results, unsigned *genomeLocations,
                    Direction *hitDirections, int *finalScores, int *mapqs);
    // BaseAligner::AlignRead(read, &loc, &dir, &score, &mapq, 0, 0, 0, maxHitsToGet, &multiHitsFound,
    // multiHitLocations, multiHitRCs, multiHitScores) (BaseAligner.h:73-86, as PairedAligner.cpp:
    // 602-605 calls it) of reads[0..n) in one GPU batch; read i's hits are at [i * maxHitsToGet, ...)
    void AlignReadsMultiHit(Read **reads, unsigned n, unsigned maxHitsToGet, AlignmentResult *results,
                            unsigned *genomeLocations, Direction *hitDirections, int *finalScores, int *mapqs,
                            int *multiHitsFound, unsigned *multiHitLocations, bool *multiHitRCs,
                            int *multiHitScores);
    _int64 perReadCalls() const { return nPerRead; }
    virtual _int64 getNHashTableLookups() const;
    virtual _int64 getLocationsScored() const;
    virtual _int64 getNHitsIgnoredBecauseOfTooHighPopularity() const;
    virtual _int64 getNReadsIgnoredBecauseOfTooManyNs() const;
    virtual _int64 getNIndelsMerged() const;
    virtual void addIgnoredReads(_int64 newlyIgnoredReads);
    virtual const char *getRCTranslationTable() const;
    virtual int getMaxK() const;
    virtual const char *getName() const;

private:
    snapgpu_aligner_stats_t stats() const;
    snapgpu_reads_t *copyReads(Read **reads, unsigned n);
    snapgpu_index_t *idx;
    snapgpu_aligner_t *gpu;
    _int64 ignoredReads;
    _int64 nPerRead;   // AlignRead calls (one-read batches)
};

class GpuSingleExtension : public AlignerExtension {
public:
    // batchReads: reads per GPU batch; device -1 = one GPU per thread, round robin
    GpuSingleExtension(unsigned batchReads = 1u << 20, int device = -1);
    virtual ~GpuSingleExtension();

    virtual void initialize();                 // loads both indexes once (AlignerContext.cpp:104)
    virtual AlignerExtension *copy();          // per-thread copy (AlignerContext.cpp:141)
    virtual void beginThread();                // GPU aligners of this thread
    virtual void finishThread();
    virtual bool runIterationThread(ReadSupplier *supplier, AlignerContext *ctx);

private:
    struct Shared;                             // indexes loaded once, shared by the thread copies
    GpuSingleExtension(Shared *shared, unsigned batchReads, int device);
    Shared *shared;
    bool owner;
    unsigned batchReads;
    int device;
    snapgpu_aligner_t *g, *t;                  // genome and transcriptome aligners of this thread
};

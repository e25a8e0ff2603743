// GpuPairedEndAligner.h -- the paired-end drop-in for SNAPLib (C++98, reference headers):
// a PairedEndAligner (PairedEndAligner.h:60-78) whose align() is ChimericPairedEndAligner::align
// over IntersectingPairedEndAligner::align (ChimericPairedEndAligner.cpp:56-126,
// IntersectingPairedEndAligner.cpp:142-753) on the MI355X, through snapgpu_paired_align_batch.
// PairedAlignerContext::runIterationThread (PairedAligner.cpp:466-482) builds the pair
// `new IntersectingPairedEndAligner(...)` + `new ChimericPairedEndAligner(...)`; a maintainer
// replaces both with one GpuPairedEndAligner of the same arguments.  alignBatch() is the form a
// batching caller (an AlignerExtension over a PairedReadSupplier) uses.
#pragma once

#include "stdafx.h"
#include "PairedEndAligner.h"
#include "Read.h"

#include "snapgpu.h"

class GpuPairedEndAligner : public PairedEndAligner {
public:
    // indexDir: the reference's on-disk index (snapgpu_index_load); arguments as
    // IntersectingPairedEndAligner + ChimericPairedEndAligner take them (PairedAligner.cpp:466-482)
    GpuPairedEndAligner(const char *indexDir, int device, unsigned maxReadSize, unsigned maxHits, unsigned maxK,
                        unsigned numSeeds, double seedCoverage, unsigned minSpacing, unsigned maxSpacing,
                        unsigned maxBigHits, unsigned extraSearchDepth, unsigned maxCandidatePoolSize,
                        bool forceSpacing);
    virtual ~GpuPairedEndAligner();

    virtual void align(Read *read0, Read *read1, PairedAlignmentResult *result);
    // n pairs in one GPU batch (the Reads are copied: a Read is only valid until the next
    // getNextReadPair, Read.h:135)
    void alignBatch(Read **reads0, Read **reads1, unsigned n, PairedAlignmentResult *results);
    virtual _int64 getLocationsScored() const;

private:
    snapgpu_index_t *idx;
    snapgpu_paired_aligner_t *gpu;
    _int64 locationsScored;
    _int64 nPerPair;   // align() calls (one-pair batches)
};

// gpu_snap_main.cpp -- apps/snap/Main.cpp's `single` command with the MI355X extension plugged
// in: the only change a SNAPLib maintainer makes to the entry point (Main.cpp:64-69 constructs
// SingleAlignerContext with no extension).
#include "stdafx.h"
#include "SingleAligner.h"
#include "exit.h"
#include "GpuSingleExtension.h"
#include "GpuPairedEndAligner.h"
#include "Read.h"

#include <fstream>
#include <string>
#include <vector>

static const char *SNAP_VERSION = "0.1alpha";

// `pairs <index-dir> <reads1.fq> <reads2.fq>`: GpuPairedEndAligner (the PairedEndAligner drop-in)
// over two FASTQ files with the paired CLI's defaults, one line per pair:
// status0 status1 loc0 loc1 dir0 dir1 score0 score1 mapq0 mapq1 fromAlignTogether alignedAsPair
static int runPairs(int argc, const char **argv)
{
    if (argc < 5) { fprintf(stderr, "usage: snap-rna-gpu pairs <index-dir> <reads1.fq> <reads2.fq>\n"); return 1; }
    GpuPairedEndAligner aligner(argv[2], 0, MAX_READ_LENGTH, 16000, 15, 8, 0, 50, 1000, 16000, 2, 1000000, false);
    std::ifstream in0(argv[3]), in1(argv[4]);
    std::string l0[4], l1[4];
    std::vector<std::string> keep;
    while (std::getline(in0, l0[0]) && std::getline(in0, l0[1]) && std::getline(in0, l0[2]) && std::getline(in0, l0[3]) &&
           std::getline(in1, l1[0]) && std::getline(in1, l1[1]) && std::getline(in1, l1[2]) && std::getline(in1, l1[3])) {
        keep.push_back(l0[1]); keep.push_back(l0[3]); keep.push_back(l1[1]); keep.push_back(l1[3]);
    }
    const size_t n = keep.size() / 4;
    Read *r0 = new Read[n + 1], *r1 = new Read[n + 1];   // Read has no const copy (Read.h)
    std::vector<Read *> p0(n), p1(n);
    for (size_t i = 0; i < n; i++) {
        r0[i].init("r", 1, keep[4 * i].c_str(), keep[4 * i + 1].c_str(), (unsigned)keep[4 * i].size());
        r1[i].init("r", 1, keep[4 * i + 2].c_str(), keep[4 * i + 3].c_str(), (unsigned)keep[4 * i + 2].size());
        p0[i] = &r0[i]; p1[i] = &r1[i];
    }
    std::vector<PairedAlignmentResult> res(n > 0 ? n : 1);
    if (n) aligner.alignBatch(&p0[0], &p1[0], (unsigned)n, &res[0]);
    for (size_t i = 0; i < n; i++) {
        const PairedAlignmentResult &r = res[i];
        printf("%d\t%d\t%u\t%u\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\n", (int)r.status[0], (int)r.status[1], r.location[0],
               r.location[1], (int)r.direction[0], (int)r.direction[1], r.score[0], r.score[1], r.mapq[0], r.mapq[1],
               (int)r.fromAlignTogether, (int)r.alignedAsPair);
    }
    delete[] r0;
    delete[] r1;
    return 0;
}

int main(int argc, const char **argv)
{
    if (argc >= 2 && strcmp(argv[1], "pairs") == 0) return runPairs(argc, argv);
    if (argc < 2 || strcmp(argv[1], "single") != 0) {
        fprintf(stderr, "usage: snap-rna-gpu single <genome-dir> <transcriptome-dir> <annotation> <reads> [options]\n"
                        "       snap-rna-gpu pairs <index-dir> <reads1.fq> <reads2.fq>\n");
        soft_exit(1);
    }
    unsigned nArgsConsumed;
    SingleAlignerContext single(new GpuSingleExtension());
    single.runAlignment(argc - 2, argv + 2, SNAP_VERSION, &nArgsConsumed);
    return 0;
}

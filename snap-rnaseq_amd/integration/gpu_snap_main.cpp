// gpu_snap_main.cpp -- apps/snap/Main.cpp's `single` command with the MI355X extension plugged
// in: the only change a SNAPLib maintainer makes to the entry point (Main.cpp:64-69 constructs
// SingleAlignerContext with no extension).
#include "stdafx.h"
#include "SingleAligner.h"
#include "exit.h"
#include "GpuSingleExtension.h"

static const char *SNAP_VERSION = "0.1alpha";

int main(int argc, const char **argv)
{
    if (argc < 2 || strcmp(argv[1], "single") != 0) {
        fprintf(stderr, "usage: snap-rna-gpu single <genome-dir> <transcriptome-dir> <annotation> <reads> [options]\n");
        soft_exit(1);
    }
    unsigned nArgsConsumed;
    SingleAlignerContext single(new GpuSingleExtension());
    single.runAlignment(argc - 2, argv + 2, SNAP_VERSION, &nArgsConsumed);
    return 0;
}

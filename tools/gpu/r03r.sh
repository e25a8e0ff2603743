#!/bin/bash
# rocprofv3 kernel trace of the RNA leg (tools/rna_probe.py: transcriptome / genome / paired aligners and
# the whole snapgpu_rna_paired_align call on 100k 2 x 150 pairs) of the current build
export TMPDIR=/tmp
mkdir -p gpurun_out/rna_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rna_prof/kt -o run --output-format csv -- python3 tools/rna_probe.py > gpurun_out/rna_prof/rna_probe.log 2> gpurun_out/rna_prof/rna_probe.err || { tail -5 gpurun_out/rna_prof/rna_probe.err; exit 1; }
tail -1 gpurun_out/rna_prof/rna_probe.log
f=$(find gpurun_out/rna_prof/kt -name "run_kernel_stats.csv" | head -1)
cp $f gpurun_out/rna_prof/kernel_stats.csv
head -12 gpurun_out/rna_prof/kernel_stats.csv | cut -c1-200

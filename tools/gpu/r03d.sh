#!/bin/bash
# round 3: PMC traffic of the variants on C2, then C3 A/B (index built once, shared) with record digests
mkdir -p gpurun_out/r03d
timeout -k 10 120 ./tools/gpu/valu_rates > gpurun_out/r03d/valu_rates.json 2>&1 || { cat gpurun_out/r03d/valu_rates.json; exit 1; }
bash tools/gpu/pmcx.sh r03d cur base || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03d/c3_build.log 2>&1 || { tail -5 gpurun_out/r03d/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for v in base cur; do
  if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03d/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03d/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03d/c3_ab.log
# RNA leg (bench extras.rna_paired workload): stage times and the kernel trace of the current build
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03d/rna_kt -o run --output-format csv -- python3 tools/rna_probe.py > gpurun_out/r03d/rna_probe.txt 2> gpurun_out/r03d/rna_probe.err || { tail -5 gpurun_out/r03d/rna_probe.err; exit 1; }
tail -3 gpurun_out/r03d/rna_probe.txt

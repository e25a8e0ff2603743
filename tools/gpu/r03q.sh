#!/bin/bash
# A/B of wave_sync as a compiler-only barrier (no s_waitcnt lgkmcnt(0) after LDS writes: one wave per
# workgroup, LDS and vector memory ops of a wave complete in order): GPU suite on the variant, then C2
# (3 alternating rounds) and C3 (2 rounds) against the current build, 2-rank self-launch rehearsal
mkdir -p gpurun_out/r03q
export SNAPGPU_TIMEOUT_S=90
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_LIB=$L/libsnapgpu_ws.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03q/gpu_tests_ws.log 2>&1 || { tail -30 gpurun_out/r03q/gpu_tests_ws.log; exit 1; }
tail -1 gpurun_out/r03q/gpu_tests_ws.log
bash tools/gpu/abx.sh r03q 3 cur ws || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03q/c3_build.log 2>&1 || { tail -5 gpurun_out/r03q/c3_build.log; exit 1; }
for i in 1 2; do for v in cur ws; do
  if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03q/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03q/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03q/c3_ab.log
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r03q/bench_2rank.json 2> gpurun_out/r03q/bench_2rank.err || { tail -5 gpurun_out/r03q/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03q/bench_2rank.json').readline()); print('2 ranks', d['n_gpus'], round(d['value']/1e6,3), [round(r['reads_per_s']/1e6,2) for r in d['config']['per_rank']])"

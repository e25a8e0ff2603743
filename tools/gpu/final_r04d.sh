#!/bin/bash
# rocprof evidence, then the final evidence run against the freshly folded pmc_traffic.json
bash tools/gpu/prof.sh r04 > gpurun_out/prof_r04.log 2>&1 || { tail -20 gpurun_out/prof_r04.log; exit 1; }
tail -1 gpurun_out/prof_r04.log
bash tools/gpu/final_r04c.sh

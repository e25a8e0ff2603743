#!/bin/bash
# summarize the last gpu_quick.sh run
tail -4 gpurun_out/t.log
python3 -c "
import json;d=json.load(open('gpurun_out/phase.log'));print(d['kernel_ms']); print({k:round(v,2) for k,v in d['cycles_per_read'].items()})" 2>/dev/null
cut -c1-200 gpurun_out/bp.log 2>/dev/null

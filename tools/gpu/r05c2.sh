#!/bin/bash
# Two RNA-leg A/Bs on one box: align_kernel<256> at 5 waves/SIMD (tools/gpu/r05w5.sh) and the host
# worker count of the RNA stages (tools/gpu/r05ht.sh).
bash tools/gpu/r05w5.sh ${1:?tag}_w5 && bash tools/gpu/r05ht.sh ${1}_ht

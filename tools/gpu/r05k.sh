#!/bin/bash
# Round 5: the RNA side-stream / two-part transcriptome call tests and sub-batch probe, then the
# lane-pair prefilter A/B with instruction counts.
bash tools/gpu/rna_sub.sh r05k && bash tools/gpu/ab_pmc.sh r05k_ab pf4 pf5 pf5w5

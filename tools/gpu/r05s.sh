#!/bin/bash
# Round 5: C2 and C3 A/B of the HBM chain-head build (cur) against the previous build (prev).
bash tools/gpu/ab_pmc.sh r05s_ab prev && bash tools/gpu/c3_ab.sh r05s_c3 prev

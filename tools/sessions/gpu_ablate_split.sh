#!/bin/bash
mkdir -p gpurun_out
export SPLIT=1
./tools/bf_ablate.sh > gpurun_out/ablate_split.log 2>&1 || { cat gpurun_out/ablate_split.log; exit 1; }
LOC=0 timeout -k 5 120 build/ablate/ablate_s_base 1000000 10000 s_base_loc0 >> gpurun_out/ablate_split.log 2>&1
SPLIT=0 timeout -k 5 120 build/ablate/ablate_s_base 1000000 10000 fp32_base >> gpurun_out/ablate_split.log 2>&1
cat gpurun_out/ablate_split.log

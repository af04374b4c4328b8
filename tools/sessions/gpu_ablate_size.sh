#!/bin/bash
# Same pair count (1e10) at corpus images of 512 / 64 / 16 MB: does a
# cache-resident corpus (MALL / L2) speed the split key pass up?
mkdir -p gpurun_out
export SPLIT=1
L=gpurun_out/ablate_size.log; : > $L
for cfg in "1000000 10000" "125000 80000" "31250 320000"; do
  timeout -k 5 90 build/ablate/ablate_s_base $cfg "size_$cfg" >> $L 2>&1 || { cat $L; exit 1; }
done
cat $L

#!/bin/bash
# Split key pass ablations (tools/bf_ablate.sh build first): query block
# 256 / 128, variants compiled with -D flags.
mkdir -p gpurun_out
export SPLIT=1
L=gpurun_out/ablate_pf.log; : > $L
for v in ${VARS:-s_base s_nosgb s_noepi s_noloads}; do
  for bq in ${BQS:-192 256}; do
    BQ=$bq timeout -k 5 60 build/ablate/ablate_$v 1000000 10000 "${v}_bq${bq}" >> $L 2>&1 || { cat $L; exit 1; }
  done
done
cat $L

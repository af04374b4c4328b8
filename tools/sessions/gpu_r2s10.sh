#!/bin/bash
# 16x16x32 key pass ablations (no-min keeps both accumulators of a column live)
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for v in base noext nomin nofill pure base; do
  timeout -k 5 120 $B/abl_$v 1000000 10000 128 q_$v || exit $?
done

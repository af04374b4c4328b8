#!/bin/bash
# 16x16x32 key pass ablations: no extraction / no minima / no barrier + fills
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for v in base noext nomin pure base; do
  timeout -k 5 120 $B/abl_$v 1000000 10000 128 q_$v || exit $?
done
timeout -k 5 120 $B/abl_noext 15625 640000 128 q_noext_l2 || exit $?
WV_H16_RUN_SEED=1 timeout -k 5 120 $B/abl_base 1000000 10000 128 q_base_runseed || exit $?
timeout -k 5 120 $B/abl_base 1000000 10000 128 q_base || exit $?

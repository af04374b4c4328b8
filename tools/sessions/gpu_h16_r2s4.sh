#!/bin/bash
# f16 key pass: extraction-code presence vs work, and corpus residency
# (HBM / MALL / L2-sized corpus image at the same pair count)
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for v in base extnever noext; do
  timeout -k 5 120 $B/abl_$v 1000000 10000 128 $v || exit $?
done
timeout -k 5 120 $B/abl_base 125000 80000 128 base_mall || exit $?
timeout -k 5 120 $B/abl_noext 125000 80000 128 noext_mall || exit $?
timeout -k 5 120 $B/abl_base 15625 640000 128 base_l2 || exit $?
timeout -k 5 120 $B/abl_noext 15625 640000 128 noext_l2 || exit $?
timeout -k 5 120 $B/abl_base 1000000 10000 128 base_again || exit $?

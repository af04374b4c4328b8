#!/bin/bash
# banded (XCD-shared corpus tiles) schedule vs one band, then the exact-path GPU tests
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for nb in 1 8 4 2 1 8; do
  WV_H16_BANDS=$nb timeout -k 5 120 $B/abl_base 1000000 10000 128 base_bands$nb || exit $?
done
WV_H16_BANDS=1 timeout -k 5 120 $B/abl_noext 1000000 10000 128 noext_bands1 || exit $?
WV_H16_BANDS=8 timeout -k 5 120 $B/abl_noext 1000000 10000 128 noext_bands8 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
   -k "h16 or bruteforce or large_k or split_pass or allow_list" > gpurun_out/r2s5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2s5_tests.log; exit $rc

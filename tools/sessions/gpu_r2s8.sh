#!/bin/bash
# 16x16x32 f16 key pass (default at D = 128) vs the 32x32x16 pass (WV_H16_QUAD=0)
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for q in 1 0 1 0; do
  WV_H16_QUAD=$q timeout -k 5 120 $B/abl_base 1000000 10000 128 quad$q || exit $?
done
WV_H16_QUAD=1 timeout -k 5 120 $B/abl_dbg 1000000 10000 128 dbg_quad || exit $?
unset WV_ABLATE_NO_FALLBACK
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread \
   -k "h16 or bruteforce or large_k or allow_list or acceptance or merge" > gpurun_out/r2s8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2s8_tests.log; exit $rc

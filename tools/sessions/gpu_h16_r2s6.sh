#!/bin/bash
# tiles per LDS stage 2 vs 3, then the exact-path GPU tests
mkdir -p gpurun_out
export WV_ABLATE_NO_FALLBACK=1
B=build/h16
for v in base tps3 base tps3; do
  timeout -k 5 120 $B/abl_$v 1000000 10000 128 $v || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread \
   -k "h16 or bruteforce or large_k or split_pass or allow_list" > gpurun_out/r2s6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2s6_tests.log; exit $rc

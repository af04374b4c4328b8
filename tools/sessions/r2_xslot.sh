#!/bin/bash
# cross-slot threshold (WV_H16_XSLOT=1) vs the seed-only default, alternated,
# then the f16 parity tests and the exact-path tests with it on
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/xslot.log
for r in 1 2; do
  for x in 0 1; do
    WV_H16_XSLOT=$x timeout -k 5 120 build/h16/abl_base 1000000 10000 128 xslot$x >> gpurun_out/xslot.log 2>&1 || exit $?
  done
done
WV_H16_XSLOT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xslot_tests.log 2>&1
rc=$?
cat gpurun_out/xslot.log; tail -n 3 gpurun_out/xslot_tests.log
exit $rc

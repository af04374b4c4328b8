#!/bin/bash
# cross-slot threshold: stores at 1/16..1/2 read back 8 tiles later (abl_base)
# vs stores at 1/8..1/2 read at the next point (abl_prev), alternated
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/xslot4.log
for r in 1 2 3; do
  timeout -k 5 120 build/h16/abl_prev 1000000 10000 128 prev >> gpurun_out/xslot4.log 2>&1 || exit $?
  timeout -k 5 120 build/h16/abl_base 1000000 10000 128 lag8 >> gpurun_out/xslot4.log 2>&1 || exit $?
done
cat gpurun_out/xslot4.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xslot4_tests.log 2>&1
rc=$?
tail -n 3 gpurun_out/xslot4_tests.log
exit $rc

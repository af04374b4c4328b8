#!/bin/bash
# cross-slot threshold with its SGPR pressure trimmed vs the default, alternated
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/xslot3.log
for r in 1 2 3; do
  WV_H16_XSLOT=0 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 xslot0 >> gpurun_out/xslot3.log 2>&1 || exit $?
  WV_H16_XSLOT=1 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 xslot1 >> gpurun_out/xslot3.log 2>&1 || exit $?
done
cat gpurun_out/xslot3.log

#!/bin/bash
# 4-wave vs 8-wave workgroups on both key-pass shapes; seed stride 12
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/waves.log
for q in 0 1; do
  for w in 8 4; do
    WV_H16_QUAD=$q WV_H16_WAVES=$w timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q${q}_w$w >> gpurun_out/waves.log 2>&1 || exit $?
  done
  WV_H16_QUAD=$q WV_H16_SAMPLE=12 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q${q}_s12 >> gpurun_out/waves.log 2>&1 || exit $?
done
cat gpurun_out/waves.log

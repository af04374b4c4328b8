#!/bin/bash
# seed pre-pass tile stride sweep (WV_H16_SAMPLE) on both key-pass shapes
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/sample.log
for q in 0 1; do
  for s in 8 16 24 32 48 64; do
    WV_H16_QUAD=$q WV_H16_SAMPLE=$s timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q${q}_s$s >> gpurun_out/sample.log 2>&1 || exit $?
  done
done
cat gpurun_out/sample.log

#!/bin/bash
# 16x16x32 key pass: what the corpus stream costs -- the DMA itself, the
# counted waits for it, or the workgroup barrier (results of the variants
# without waits / barrier are garbage; only their time is read)
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fillsync.log
for v in base novmwait nobarrier nosync nofill base; do
  WV_ABLATE_NO_FALLBACK=1 WV_H16_QUAD=1 timeout -k 5 120 build/h16/abl_$v 1000000 10000 128 q_$v >> gpurun_out/fillsync.log 2>&1 || exit $?
done
cat gpurun_out/fillsync.log

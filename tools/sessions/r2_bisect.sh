#!/bin/bash
# 16x16x32 key pass, everything but the MFMA/LDS loop compiled out, then the
# tile bookkeeping (tile_ok) and the counted DMA waits removed as well
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bisect.log
for v in base pure pure_notileok pure_novmwait pure_both; do
  WV_ABLATE_NO_FALLBACK=1 WV_H16_QUAD=1 timeout -k 5 120 build/h16/abl_$v 1000000 10000 128 q_$v >> gpurun_out/bisect.log 2>&1 || exit $?
done
cat gpurun_out/bisect.log

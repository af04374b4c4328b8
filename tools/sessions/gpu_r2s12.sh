#!/bin/bash
# 8-wave vs two 4-wave workgroups per CU (16x16x32 key pass), then the full
# GPU suite + smoke + bench + rocprof stats, then the key-pass PMC passes
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 8 4 8 4; do
  WV_ABLATE_NO_FALLBACK=1 WV_H16_WAVES=$w timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q_waves$w > /dev/null 2>&1
  WV_ABLATE_NO_FALLBACK=1 WV_H16_WAVES=$w timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q_waves$w \
      >> gpurun_out/r2s12_waves.log 2>&1 || exit $?
done
cat gpurun_out/r2s12_waves.log
TAG=r2s12 bash tools/gpu_r2_full.sh || exit $?
N=1000000 NQ=10000 D=128 B=build/h16/abl_base timeout -k 10 300 bash tools/pmc_h16.sh > gpurun_out/r2s12_pmc.log 2>&1
echo "pmc rc=$?"

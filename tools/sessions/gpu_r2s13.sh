#!/bin/bash
# default (32x32x16) vs WV_H16_QUAD=1 with true fallback counts, then the
# default bench + rocprof stats (no tests: r2s12 ran the suite), then PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
for q in 0 1; do
  WV_ABLATE_NO_FALLBACK=1 WV_H16_QUAD=$q timeout -k 5 120 build/h16/abl_base 1000000 10000 128 quad$q \
      >> gpurun_out/r2s13_quad.log 2>&1 || exit $?
done
cat gpurun_out/r2s13_quad.log
NO_TESTS=1 TAG=r2s13 bash tools/gpu_r2_full.sh || exit $?
N=1000000 NQ=10000 D=128 B=build/h16/abl_base timeout -k 10 300 bash tools/pmc_h16.sh > gpurun_out/r2s13_pmc.log 2>&1
echo "pmc rc=$?"

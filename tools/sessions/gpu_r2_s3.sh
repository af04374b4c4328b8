#!/bin/bash
# round-2 session 3: f16 key-pass variant timings (harness), then the full
# GPU suite, smoke, the default bench and its rocprof stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 bash tools/h16_ablate.sh > gpurun_out/r2s3_h16_variants.log 2>&1
rc=$?; echo "ablate rc=$rc"; cat gpurun_out/r2s3_h16_variants.log
case $rc in 124|134|137|139) exit $rc;; esac
TAG=r2s3 bash tools/gpu_r2_full.sh

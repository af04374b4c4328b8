#!/bin/bash
# 16x16x32 key pass with shared 16-entry column lists vs the 32x32x16 default,
# then the GPU suite with the 16x16x32 kernel forced on
export TMPDIR=/tmp
mkdir -p gpurun_out
WV_H16_QUAD=0 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 quad0 > gpurun_out/qc.log 2>&1 &&
WV_H16_QUAD=1 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 quad1 >> gpurun_out/qc.log 2>&1 &&
WV_H16_QUAD=1 WV_H16_NO_SEED=1 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 quad1_noseed >> gpurun_out/qc.log 2>&1 &&
WV_H16_QUAD=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qc_tests.log 2>&1
rc=$?
cat gpurun_out/qc.log; tail -5 gpurun_out/qc_tests.log
exit $rc

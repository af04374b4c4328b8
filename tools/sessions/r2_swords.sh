#!/bin/bash
# tile eligibility words by scalar loads: key pass on both shapes, then the
# GPU suite on the default shape and on the 16x16x32 one
export TMPDIR=/tmp
mkdir -p gpurun_out
WV_H16_QUAD=0 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q0_swords > gpurun_out/swords.log 2>&1 &&
WV_H16_QUAD=1 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q1_swords >> gpurun_out/swords.log 2>&1 &&
WV_H16_QUAD=0 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q0_swords >> gpurun_out/swords.log 2>&1 &&
WV_H16_QUAD=1 timeout -k 5 120 build/h16/abl_base 1000000 10000 128 q1_swords >> gpurun_out/swords.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/swords_tests.log 2>&1 &&
WV_H16_QUAD=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/swords_tests_q.log 2>&1
rc=$?
cat gpurun_out/swords.log; tail -3 gpurun_out/swords_tests.log gpurun_out/swords_tests_q.log
exit $rc

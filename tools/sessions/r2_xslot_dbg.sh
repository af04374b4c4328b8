#!/bin/bash
# extraction rounds with and without the cross-slot threshold (debug
# counters build), and the seed stride 8 for comparison
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/xslot_dbg.log
WV_H16_XSLOT=0 timeout -k 5 120 build/h16/abl_dbg 1000000 10000 128 dbg_x0 >> gpurun_out/xslot_dbg.log 2>&1 &&
WV_H16_XSLOT=1 timeout -k 5 120 build/h16/abl_dbg 1000000 10000 128 dbg_x1 >> gpurun_out/xslot_dbg.log 2>&1 &&
WV_H16_SAMPLE=8 timeout -k 5 120 build/h16/abl_dbg 1000000 10000 128 dbg_s8 >> gpurun_out/xslot_dbg.log 2>&1
rc=$?
cat gpurun_out/xslot_dbg.log
exit $rc

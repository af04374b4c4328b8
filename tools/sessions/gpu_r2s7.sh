#!/bin/bash
# bare f16 MFMA shapes (32x32x16 vs 16x16x32), then the key pass's extraction counters
mkdir -p gpurun_out
timeout -k 5 60 build/mfma_shape_bench 20000 || exit $?
export WV_ABLATE_NO_FALLBACK=1
timeout -k 5 120 build/h16/abl_dbg 1000000 10000 128 dbg || exit $?
WV_H16_NO_SEED=1 timeout -k 5 120 build/h16/abl_dbg 1000000 10000 128 dbg_noseed || exit $?

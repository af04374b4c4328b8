#!/bin/bash
# BASELINE configs[2] exact line only (GloVe-100-shaped 1.2M x 100 cosine):
# D = 100 -> stride 128, the bf16x3 split pass.
mkdir -p gpurun_out
B="--rows 1200000 --dim 100 --metric cosine-dot --data gauss --nq 10000"
timeout -k 10 400 python -u bench.py $B --cpu-seconds 8 > gpurun_out/c3_exact.log 2>&1 || exit $?
tail -1 gpurun_out/c3_exact.log | cut -c1-1600

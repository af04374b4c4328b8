#!/bin/bash
# C5 shard: one GPU's share of the 100M x 96 L2 corpus sharded 8-way
# (12.5M rows), graph built on the GPU (M=64, efC=128), HNSW, 10k queries.
mkdir -p gpurun_out
for ef in ${EFS:-64}; do
  timeout -k 10 600 python -u bench.py --workload hnsw --rows ${ROWS:-12500000} --dim 96 --data sift \
    --graph-build gpu --ef $ef --cpu-seconds 10 > gpurun_out/bench_c5_ef$ef.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_c5_ef$ef.log
done

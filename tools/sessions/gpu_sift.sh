#!/bin/bash
# C1 (BASELINE configs[0]): 1M x 128 SIFT-shaped L2, M=64 efC=128, graph built
# once by the CPU restatement (cached for this call), ef sweep; then the same
# data with the graph built on the GPU; then rocprofv3 passes at ef=64.
mkdir -p gpurun_out
CACHE=/tmp/wv_graph_sift_1m.npz
A="--workload hnsw --data sift"
for ef in 64 32 128 256; do
  timeout -k 10 900 python -u bench.py $A --ef $ef --graph-cache $CACHE --steps 3 --warmup 1 --cpu-seconds 8 \
      > gpurun_out/sift_ef$ef.log 2>&1 || exit $?
  tail -1 gpurun_out/sift_ef$ef.log | cut -c1-400
done
timeout -k 10 600 python -u bench.py $A --graph-build gpu --steps 3 --warmup 1 --cpu-seconds 8 \
    > gpurun_out/sift_gpubuild.log 2>&1 || exit $?
BENCH_ARGS="$A --ef 64 --graph-cache $CACHE --no-cpu-baseline --steps 3 --warmup 1" bash tools/profile.sh ${TAG:-r01_sift}

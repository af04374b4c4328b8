#!/bin/bash
# HNSW bench at scale + rocprofv3 passes; the graph is built once by the CPU
# restatement and cached in /tmp for the profile passes of the same call.
mkdir -p gpurun_out
N=${HN:-1000000}
TAG=${TAG:-r01_hnsw}
CACHE=/tmp/wv_graph_${N}.npz
ARGS="--workload hnsw --rows $N --ef ${EF:-64} --graph-cache $CACHE"
timeout -k 10 1000 python -u bench.py $ARGS --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_hnsw.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_hnsw.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="$ARGS --no-cpu-baseline --steps 3 --warmup 1" bash tools/profile.sh $TAG

#!/bin/bash
# 1M x 128 HNSW: graph built on the GPU (wv_index_build_graph), searched, CPU leg
# searching the same graph.  Then the C3-shaped cosine build.
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload hnsw --graph-build gpu --batch-div ${DIV:-64} \
    --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_hnsw_gpubuild.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_hnsw_gpubuild.log | cut -c1-3000
exit $rc

#!/bin/bash
# HNSW speculative neighbour prefetch: GPU parity tests (hnsw / graph / pq),
# then C1 SIFT-shaped 1M x 128 with the graph built on the GPU, ef 64 and 128.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu -k "hnsw or graph or kat or pq or mutable or batcher" --timeout 180 --timeout-method thread > gpurun_out/tests_hnsw.log 2>&1
rc=$?; tail -3 gpurun_out/tests_hnsw.log; [ $rc -eq 0 ] || exit $rc
for ef in 64 128; do
  timeout -k 10 600 python -u bench.py --workload hnsw --data sift --graph-build gpu --ef $ef --cpu-seconds 6 > gpurun_out/spec_ef$ef.log 2>&1 || exit $?
  tail -1 gpurun_out/spec_ef$ef.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity_sample']; r=d['roofline']; print('ef=$ef', d['value'], r['kernel_ms'], r['frac'], r['gpu_dist_evals_per_query'], p['recall@10_gpu'], p['recall@10_cpu_restatement'], p['tie_aware_identical_frac'], d['graph']['build_s'])"
done

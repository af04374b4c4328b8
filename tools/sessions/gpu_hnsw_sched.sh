#!/bin/bash
# A/B of the HNSW locality schedule (WV_HNSW_NO_SORT=1 disables it) on C1
# SIFT-shaped and uniform data, graphs built on the GPU; parity tests first.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_pq.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hnsw or build or compressed" > gpurun_out/sched_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sched_tests.log; [ $rc -eq 0 ] || exit $rc
for data in sift uniform; do
  for ns in 1 0; do
    if [ $ns = 1 ]; then export WV_HNSW_NO_SORT=1; else unset WV_HNSW_NO_SORT; fi
    timeout -k 10 600 python -u bench.py --workload hnsw --data $data --graph-build gpu --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sched_${data}_nosort$ns.log 2>&1 || exit $?
    python3 -c "
import json;r=json.loads(open('gpurun_out/sched_${data}_nosort$ns.log').read().strip().splitlines()[-1])
print('$data nosort=$ns', r['value'], r['ms_per_step'], r['roofline']['kernel_ms'], r['roofline']['frac'])"
  done
done

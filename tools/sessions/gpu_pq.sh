mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pq.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pq_tests.log 2>&1
rc=$?; tail -25 gpurun_out/pq_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hnsw or build" > gpurun_out/hnsw_tests.log 2>&1
rc=$?; tail -5 gpurun_out/hnsw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload hnsw --graph-build gpu --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sift_after_pq.log 2>&1
rc=$?; tail -1 gpurun_out/sift_after_pq.log | cut -c1-600; exit $rc

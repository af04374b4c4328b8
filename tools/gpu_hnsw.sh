#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "hnsw or kat" --timeout 180 --timeout-method thread > gpurun_out/tests_hnsw.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests_hnsw.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --workload hnsw --n ${HN:-200000} --ef 64 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_hnsw.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_hnsw.log | cut -c1-3000

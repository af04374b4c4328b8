#!/bin/bash
# exact-path tests after the fused qnorm/absmax kernel, then the bench (no CPU baseline)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide_k.py tests/test_gpu_wide_d.py tests/test_gpu_async.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2s14_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2s14_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-hnsw-line > gpurun_out/r2s14_bench.jsonl 2> gpurun_out/r2s14_bench.err
rc=$?; cut -c1-900 gpurun_out/r2s14_bench.jsonl; exit $rc

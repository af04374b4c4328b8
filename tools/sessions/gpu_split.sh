#!/bin/bash
# bf16x3 key pass: the brute-force parity tests, then the configs[1] bench with
# the split pass and with the fp32 MFMA pass (WV_BF_FP32=1).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; tail -4 gpurun_out/split_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/split_bench.log 2>&1 || exit $?
tail -1 gpurun_out/split_bench.log | cut -c1-1500
WV_BF_FP32=1 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fp32_bench.log 2>&1 || exit $?
tail -1 gpurun_out/fp32_bench.log | cut -c1-700

#!/bin/bash
# Native-image split kernel: parity tests, configs[1] bench, ablation harness.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nat_tests.log 2>&1
rc=$?; tail -15 gpurun_out/nat_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/nat_bench.log 2>&1 || exit $?
tail -1 gpurun_out/nat_bench.log | cut -c1-1600
SPLIT=1 ./tools/bf_ablate.sh > gpurun_out/nat_ablate.log 2>&1; cat gpurun_out/nat_ablate.log

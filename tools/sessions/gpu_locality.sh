#!/bin/bash
# Brute-force schedule locality: parity tests, then the configs[1] bench with
# WV_BF_LOCALITY = 3 (default), 1, 2, 0 and the kernel trace of the default.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/loc_tests.log 2>&1
rc=$?; tail -4 gpurun_out/loc_tests.log; [ $rc -eq 0 ] || exit $rc
for L in 3 0 1 2; do
  WV_BF_LOCALITY=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/loc_bench_$L.log 2>&1 || exit $?
  echo "L=$L $(tail -1 gpurun_out/loc_bench_$L.log | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ')"
done

#!/bin/bash
# Split key pass: 256-query blocks (one 512-thread workgroup per CU) vs the
# 128-query two-workgroup variant; exact parity tests first.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "exact or split or bf" --timeout 120 --timeout-method thread > gpurun_out/tests_bq.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tests_bq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_bq256.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bq256.log
WV_BF_BQ=128 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_bq128.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bq128.log

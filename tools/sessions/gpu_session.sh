#!/bin/bash
# One GPU session: parity tests, then the default bench.  Stops at the first
# fault / abort / timeout (exit codes other than 0 or a plain test failure).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc

#!/bin/bash
# One GPU session: parity tests, the default bench (with CPU baseline), then
# rocprofv3 kernel-trace/stats + PMC passes over a short bench (tools/profile.sh).
# Stops at the first fault / abort / timeout.
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh $TAG

#!/bin/bash
# GPU session: -m gpu tests, then the default bench (unless a test step hung,
# faulted or was killed: then nothing more touches the GPU in this call).
mkdir -p gpurun_out
KARGS=()
[ -n "$TEST_K" ] && KARGS=(-k "$TEST_K")
timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${KARGS[@]}" \
    > gpurun_out/r2_gputests.log 2>&1
rc=$?
echo "tests rc=$rc" | tee -a gpurun_out/r2_gputests.log
case $rc in 124|134|137|139) exit $rc;; esac
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_LIMIT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/r2_bench.jsonl 2> gpurun_out/r2_bench.err
brc=$?
echo "bench rc=$brc"
exit $((rc > 0 ? rc : brc))

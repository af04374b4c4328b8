#!/bin/bash
# Round-2 GPU session: every -m gpu test, smoke, the default bench line, then
# rocprofv3 --kernel-trace --stats of the same bench (no CPU baseline leg).
# Any step that times out / faults / aborts ends the call.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
stop() { case $1 in 124|134|137|139) echo "stopping after rc=$1"; exit $1;; esac; }
KARGS=()
[ -n "$TEST_K" ] && KARGS=(-k "$TEST_K")
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-480} python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${KARGS[@]}" \
      > gpurun_out/${TAG}_gputests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gputests.log; stop $rc
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; stop $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-360} python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.jsonl; stop $rc
fi
if [ -z "$NO_PROF" ]; then
  timeout -k 10 ${PROF_LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run \
      -- python3 -u bench.py --no-cpu-baseline ${PROF_ARGS} > gpurun_out/${TAG}_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; stop $rc
fi
exit 0

#!/bin/bash
# End-of-round evidence on one MI355X: the whole -m gpu suite, smoke(), the
# default bench line, and a rocprofv3 kernel trace + stats of the same bench
# (no CPU baseline under the profiler).  Outputs under gpurun_out/final/.
# FINAL_SKIP_TESTS=1: the bench and profile only.
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
if [ -z "$FINAL_SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/gputests.log 2>&1; rc=$?
tail -3 $O/gputests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 300 $O/bench.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
# (the per-dispatch trace is tens of MiB: keep the stats, gzip the trace)
gzip -f $O/prof/run_kernel_trace.csv; ls -la $O/prof
echo done

#!/bin/bash
# One GPU session (gpurun): the steps named on the command line, each under
# its own time limit, stopping at the first failure.  Logs go to gpurun_out/.
#   tests:<pytest args>   python -m pytest ... (-m gpu implied by the files)
#   env:<VAR=val,...>     environment for the following steps
#   h16:<variant>:<tag>   the f16 key-pass harness at 1M x 10k (build/h16/abl_<variant>)
#   bench:<tag>:<args>    python bench.py <args>
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}
  case $kind in
    env) IFS=',' read -ra kv <<< "$rest"; for x in "${kv[@]}"; do export "$x"; done; echo "env $rest";;
    unenv) IFS=',' read -ra kv <<< "$rest"; for x in "${kv[@]}"; do unset "$x"; done; echo "unenv $rest";;
    tests) lg=gpurun_out/tests_$(date +%s).log
           eval "timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $rest" > $lg 2>&1 \
             || { echo "tests failed: $rest"; tail -30 $lg; exit 1; }; echo "tests ok: $rest"; tail -1 $lg;;
    h16) var=${rest%%:*}; tag=${rest#*:}
         WV_ABLATE_NO_FALLBACK=1 timeout -k 10 120 build/h16/abl_$var ${N:-1000000} ${NQ:-10000} ${D:-128} $tag \
             >> gpurun_out/h16.log 2>&1 || { echo "h16 failed: $rest"; exit 1; }; tail -2 gpurun_out/h16.log;;
    bench) tag=${rest%%:*}; args=${rest#*:}; [ "$args" == "$rest" ] && args=""
           timeout -k 10 400 python bench.py $args > gpurun_out/bench_$tag.log 2>&1 || { echo "bench failed: $tag"; exit 1; }
           tail -c 600 gpurun_out/bench_$tag.log; echo;;
    *) echo "unknown step $step"; exit 2;;
  esac
done

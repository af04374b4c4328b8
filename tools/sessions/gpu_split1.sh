#!/bin/bash
# one-wave-per-SIMD split kernel vs the two-wave kernel: exact parity tests
# first, then harness timing and the default bench.
mkdir -p gpurun_out
export SPLIT=1
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "split or bruteforce or exact or c4" --timeout 120 --timeout-method thread > gpurun_out/tests_split1.log 2>&1
rc=$?; tail -3 gpurun_out/tests_split1.log; [ $rc -eq 0 ] || exit $rc
L=gpurun_out/split1.log; : > $L
WV_BF_SPLIT_1W=1 BQ=256 timeout -k 5 60 build/ablate/ablate_s_base 1000000 10000 split1 >> $L 2>&1 || { cat $L; exit 1; }
BQ=256 timeout -k 5 60 build/ablate/ablate_s_base 1000000 10000 split2w >> $L 2>&1 || { cat $L; exit 1; }
cat $L
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_split1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_split1.log | cut -c1-900

#!/bin/bash
# HNSW f16 prefilter: full GPU suite, then the C1 HNSW line with and without it
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2s15_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2s15_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1 0; do
  if [ $v = 1 ]; then export WV_HNSW_NO_H16=1; else unset WV_HNSW_NO_H16; fi
  timeout -k 10 240 python -u bench.py --workload hnsw --no-cpu-baseline >> gpurun_out/r2s15_hnsw.jsonl 2>> gpurun_out/r2s15_hnsw.err || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r2s15_hnsw.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["value"], d["ms_per_step"], d["recall@10"], r["kernel_ms"], r.get("gpu_dist_evals_per_query"), r.get("dist_evals_per_query"))
PY

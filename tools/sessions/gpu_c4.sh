#!/bin/bash
# One rank's share of BASELINE configs[3] (10M x 768 dot over 8 GPUs = 1.25M rows
# per GPU), 1000-query batches, shared allow list at 1/10/50 % and none.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
A="--rows 1250000 --dim 768 --metric dot --data gauss --nq 1000 --steps 5 --warmup 2 --cpu-seconds 8"
for p in 0.01 0.1 0.5 0; do
  timeout -k 10 400 python -u bench.py $A --allow-frac $p > gpurun_out/c4_$p.log 2>&1 || exit $?
  tail -1 gpurun_out/c4_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('p=$p', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['fallback_queries'], d.get('parity_sample'), d.get('cpu_baseline',{}).get('value'))"
done

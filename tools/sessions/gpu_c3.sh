#!/bin/bash
# BASELINE configs[2]: GloVe-100-shaped 1.2M x 100 cosine (N(0,1) then
# normalized), exact line + HNSW ef sweep 32..256 on one graph (built once).
mkdir -p gpurun_out
B="--rows 1200000 --dim 100 --metric cosine-dot --data gauss --nq 10000"
timeout -k 10 400 python -u bench.py $B --steps 3 --warmup 1 --cpu-seconds 8 > gpurun_out/c3_exact.log 2>&1 || exit $?
tail -1 gpurun_out/c3_exact.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['fallback_queries'], d.get('parity_sample'), d.get('cpu_baseline',{}).get('value'))"
for ef in 32 64 128 256; do
  timeout -k 10 900 python -u bench.py $B --workload hnsw --ef $ef --graph-cache /tmp/g_c3.npz --steps 3 --warmup 1 --cpu-seconds 4 > gpurun_out/c3_ef$ef.log 2>&1 || exit $?
  tail -1 gpurun_out/c3_ef$ef.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity_sample']; print('ef=$ef', d['value'], d['ms_per_step'], d['roofline']['frac'], p['recall@10_gpu'], p['recall@10_cpu_restatement'], p['tie_aware_identical_frac'], d['cpu_baseline']['value'])"
done

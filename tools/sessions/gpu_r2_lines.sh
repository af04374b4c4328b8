#!/bin/bash
# Secondary bench lines of round 2 (one GPU): C4 share (1.25M x 768 dot, 1000
# queries, allow 0/1/10/50 %) and C3 exact (1.2M x 100 cosine, 10k queries).
mkdir -p gpurun_out
O=gpurun_out/r2_lines.jsonl; : > $O
COMMON="--no-hnsw-line --no-wide-line --cpu-seconds 3 --cpu-seconds-t1 1"
for a in 0 0.01 0.1 0.5; do
  timeout -k 10 200 python -u bench.py --rows 1250000 --dim 768 --metric dot --data gauss --nq 1000 --allow-frac $a $COMMON >> $O 2>> gpurun_out/r2_lines.err || exit $?
done
timeout -k 10 200 python -u bench.py --rows 1200000 --dim 100 --metric cosine-dot --data gauss --nq 10000 $COMMON >> $O 2>> gpurun_out/r2_lines.err || exit $?

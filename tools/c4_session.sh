#!/bin/bash
# configs[3] shard lines (1.25M x 768 dot = one GPU's 1/8 of 10M, 1000-query
# batch, shared allow list p = 0 / 50 / 10 / 1 %): bench line, then rocprofv3
# kernel trace + stats of the same run; PMC of the key pass for p = 0.
# Outputs under gpurun_out/c4/.
export TMPDIR=/tmp
O=gpurun_out/c4; mkdir -p $O
A="--rows 1250000 --dim 768 --metric dot --nq 1000 --data gauss --no-hnsw-line --no-c3-line --no-wide-line --steps 5 --warmup 2"
for p in ${PS:-0 0.5 0.1 0.01}; do
  timeout -k 10 300 python3 -u bench.py $A --allow-frac $p --cpu-seconds 6 --cpu-seconds-t1 3 > $O/bench_$p.jsonl 2> $O/bench_$p.err || { echo "bench $p failed"; exit 1; }
  tail -c 400 $O/bench_$p.jsonl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$p -o run -- python3 -u bench.py $A --allow-frac $p --no-cpu-baseline > $O/prof_$p.log 2>&1 || { echo "prof $p failed"; exit 1; }
done
if [ -n "$PMC" ]; then
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o run -- python3 -u bench.py $A --allow-frac 0 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || echo "pmc sq rc=$?"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_fetch -o run -- python3 -u bench.py $A --allow-frac 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || echo "pmc fetch rc=$?"
fi
exit 0

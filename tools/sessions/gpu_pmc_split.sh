#!/bin/bash
# Split key pass: ablation floor + PMC passes on the harness (one kernel per run).
mkdir -p gpurun_out/pmc_split
export SPLIT=1 TMPDIR=/tmp
L=gpurun_out/pmc_split/ablate.log; : > $L
for v in s_base s_noboth s_noloads s_noepi; do
  timeout -k 5 60 build/ablate/ablate_$v 1000000 10000 $v >> $L 2>&1 || { cat $L; exit 1; }
done
cat $L
B=build/ablate/ablate_s_base
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_split/p$i -o run -- $B 1000000 10000 pmc$i > gpurun_out/pmc_split/p$i.log 2>&1 || echo "pass $i failed rc=$?"
done
echo done

#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then PMC counters in
# separate passes (never combined with tracing).  Outputs: gpurun_out/prof_<tag>/.
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 3 --warmup 1"}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1
echo done

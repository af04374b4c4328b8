#!/bin/bash
# end-of-round evidence: full GPU suite, smoke, default bench (with CPU
# baselines), rocprof stats of the same bench, PMC of the key pass
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r2fin bash tools/gpu_r2_full.sh || exit $?
N=1000000 NQ=10000 D=128 B=build/h16/abl_base timeout -k 10 300 bash tools/pmc_h16.sh > gpurun_out/r2fin_pmc.log 2>&1
echo "pmc rc=$?"

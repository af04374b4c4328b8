#!/bin/bash
# full GPU suite + smoke + bench + rocprof stats, then the key-pass PMC passes
set -o pipefail
TAG=r2s11 bash tools/gpu_r2_full.sh || exit $?
N=1000000 NQ=10000 D=128 B=build/h16/abl_base timeout -k 10 300 bash tools/pmc_h16.sh > gpurun_out/r2s11_pmc.log 2>&1
echo "pmc rc=$?"

#!/bin/bash
mkdir -p gpurun_out
SPLIT=1 ./tools/bf_ablate.sh > gpurun_out/nat_ablate.log 2>&1; rc=$?; cat gpurun_out/nat_ablate.log; exit $rc

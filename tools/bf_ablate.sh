#!/bin/bash
# Build kernel variants on the CPU side (before gpurun) and time them on the GPU.
# Variants: name=defines pairs in VARIANTS.
set -e
B=build/ablate; mkdir -p $B
HF="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off"
VARIANTS=${VARIANTS:-"w2=-DWV_BF_WAVES_PER_SIMD=2 w1=-DWV_BF_WAVES_PER_SIMD=1 w2_noepi=-DWV_BF_WAVES_PER_SIMD=2:-DWV_BF_ABLATE_NO_EPILOGUE w1_noepi=-DWV_BF_WAVES_PER_SIMD=1:-DWV_BF_ABLATE_NO_EPILOGUE"}
if [ "$1" == "build" ]; then
  /opt/rocm/bin/hipcc $HF -x hip -c tools/bf_ablate.cpp -o $B/main.o 2>/dev/null
  rm -f $B/ablate_*
  for v in $VARIANTS; do
    name=${v%%=*}; defs=${v#*=}; defs=${defs//:/ }
    /opt/rocm/bin/hipcc $HF $defs -c weaviate_amd/csrc/wv_bf.hip -o $B/bf_$name.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $B/main.o $B/bf_$name.o -o $B/ablate_$name
  done
  exit 0
fi
for f in $B/ablate_*; do
  for nb in ${BLOCKS_LIST:-512}; do
    BLOCKS=$nb timeout -k 5 120 $f ${N:-1000000} ${NQ:-10000} ${f##*/ablate_} || exit $?
  done
done

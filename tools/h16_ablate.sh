#!/bin/bash
# f16 key pass ablations: `tools/h16_ablate.sh build` (CPU side) compiles one
# harness binary per variant (name=define:define ...); without arguments (GPU
# side) runs each, plus the default binary with the seed pass off.
set -e
B=build/h16; mkdir -p $B
C=weaviate_amd/csrc
HF="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off"
VARIANTS=${VARIANTS:-"base= noext=-DWV_H16_ABLATE_NO_EXTRACT pure=-DWV_H16_ABLATE_NO_EXTRACT:-DWV_H16_ABLATE_NO_MIN:-DWV_H16_ABLATE_NO_BARRIER:-DWV_H16_ABLATE_NO_FILL"}
if [ "$1" == "build" ]; then
  make -s -C $C ARCH=gfx950
  /opt/rocm/bin/hipcc $HF -x hip -c tools/h16_ablate.cpp -o $B/main.o
  # (the API with the ablation-only fallback skip: WV_ABLATE_NO_FALLBACK)
  /opt/rocm/bin/hipcc $HF -DWV_ABLATION_BUILD -c $C/wv_api.hip -o $B/api.o
  rm -f $B/abl_*
  for v in $VARIANTS; do
    name=${v%%=*}; defs=${v#*=}; defs=${defs//:/ }
    (
    # the variant's defines apply to wv_h16.hip (the library's object without any)
    if [ -z "$defs" ]; then cp $C/wv_h16.o $B/h16_$name.o; else
      /opt/rocm/bin/hipcc $HF -fno-honor-nans $defs -c $C/wv_h16.hip -o $B/h16_$name.o; fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -pthread $B/main.o $B/h16_$name.o $C/wv_bf.o $C/wv_hnsw.o $C/wv_pq.o \
        $B/api.o $C/wv_batcher.o $C/wv_commitlog.o $C/wv_group.o $C/wv_mirror.o -L/opt/rocm/lib -lrccl -o $B/abl_$name
    ) &
  done
  wait
  exit 0
fi
export WV_ABLATE_NO_FALLBACK=1
for f in $B/abl_*; do
  timeout -k 5 120 $f ${N:-1000000} ${NQ:-10000} ${D:-128} ${f##*/abl_}
done
WV_H16_NO_SEED=1 timeout -k 5 120 $B/abl_base ${N:-1000000} ${NQ:-10000} ${D:-128} base_noseed
WV_H16_NO_RUNNING=1 timeout -k 5 120 $B/abl_base ${N:-1000000} ${NQ:-10000} ${D:-128} base_norunning


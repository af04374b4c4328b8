#!/bin/bash
# HNSW per-expansion latency: `tools/hnsw_latency.sh build` (CPU side) compiles
# one harness binary per variant (name=define:define ...); without arguments
# (GPU side) runs each.  Output: gpurun_out/hnsw_lat/<variant>.log
set -e
B=build/hnsw; mkdir -p $B
C=weaviate_amd/csrc
HF="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off"
VARIANTS=${VARIANTS:-"base= stamps=-DWV_HNSW_STAMPS rpg8=-DWV_HNSW_RPG=8 stamps8=-DWV_HNSW_STAMPS:-DWV_HNSW_RPG=8"}
if [ "$1" == "build" ]; then
  make -s -C $C ARCH=gfx950
  /opt/rocm/bin/hipcc $HF -fopenmp -x hip -c tools/hnsw_latency.cpp -o $B/main.o
  rm -f $B/lat_*
  for v in $VARIANTS; do
    name=${v%%=*}; defs=${v#*=}; defs=${defs//:/ }
    (
    if [ -z "$defs" ]; then cp $C/wv_hnsw.o $B/hnsw_$name.o; else
      /opt/rocm/bin/hipcc $HF $defs -c $C/wv_hnsw.hip -o $B/hnsw_$name.o; fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -fopenmp -pthread $B/main.o $B/hnsw_$name.o $C/wv_bf.o $C/wv_h16.o $C/wv_pq.o \
        $C/wv_api.o $C/wv_batcher.o $C/wv_commitlog.o $C/wv_group.o $C/wv_mirror.o -L/opt/rocm/lib -lrccl -o $B/lat_$name
    ) &
  done
  wait
  exit 0
fi
O=gpurun_out/hnsw_lat; mkdir -p $O
for f in $B/lat_*; do
  v=${f##*/lat_}
  timeout -k 10 240 $f ${N:-1000000} ${D:-128} $v > $O/$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/$v.log; exit 1; }
  cat $O/$v.log
done

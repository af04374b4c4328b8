#!/bin/bash
# A/B build of libwvgpu.so with extra defines (measurement infrastructure):
#   tools/ab_build.sh NAME "-DWV_HNSW_SIDE_RPG=3 ..."  ->  ab/NAME/libwvgpu.so
# loaded instead of the in-tree library when WV_LIBPATH points at it.
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/ab_build_$NAME
rm -rf $B && mkdir -p $B/weaviate_amd $B/include
cp -r $ROOT/weaviate_amd/csrc $B/weaviate_amd/ && cp $ROOT/include/*.h $B/include/
rm -f $B/weaviate_amd/csrc/*.o
make -s -j8 -C $B/weaviate_amd/csrc ARCH=gfx950 \
  HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function $DEFS"
mkdir -p $ROOT/ab/$NAME && cp $B/weaviate_amd/libwvgpu.so $ROOT/ab/$NAME/
echo "ab/$NAME/libwvgpu.so"

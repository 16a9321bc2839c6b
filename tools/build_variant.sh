#!/bin/bash
# Build a variant of the library with extra defines into fslr_amd/libfslr_hip_<name>.so (scratch tree).
# Usage: tools/build_variant.sh NAME "-DFOO -DBAR" [DIR holding replacement sources copied over csrc/]
set -e
NAME=$1; DEFS=$2; OVER=$3
ROOT=$(cd $(dirname $0)/.. && pwd)
W=/tmp/fslr_variant_$NAME
rm -rf $W && mkdir -p $W/fslr_amd && cp -r $ROOT/fslr_amd/csrc $W/fslr_amd/csrc && ln -s $ROOT/include $W/include
[ -n "$OVER" ] && cp $OVER/* $W/fslr_amd/csrc/
cd $W/fslr_amd/csrc && rm -rf *.o prof && make -s -j8 OUT=$ROOT/fslr_amd/libfslr_hip_$NAME.so \
  HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -fno-gpu-rdc -I../../include $DEFS" \
  $ROOT/fslr_amd/libfslr_hip_$NAME.so
echo built $ROOT/fslr_amd/libfslr_hip_$NAME.so
